// tools/ablate.hip -- kernel ablation / roofline harness (timing only, not part of the library).
//
// Runs the volume-sized kernels of the path on a synthetic boundary map already in HBM and times
// each variant with HIP events over `iters` launches:
//   copy_read / copy_write   plain float4 streaming read / 16-B uint64 store (the box's HBM ceiling)
//   k_block_stats            per-block min/max pass
//   k_pass1 ABL=1,2,3,0      stop after: load+threshold+bits | + tile CCL | + first voxels | full
//   k_sample_guess / k_spec  speculative front (guess = exact parameters: no relabelling)
//   k_seams STOP variants    staged faces | + the three seams | full (edges, corners)
//   k_pass2                  relabel + uint64 write (FIN = 0: timing only)
// Build: make -C tools ablate   Run: tools/ablate Z Y X bz by bx [mode] [iters]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../cluster_tools_amd/csrc/cc_kernels.hip"
#include "../cluster_tools_amd/csrc/cc_generate.hip"
#include "../cluster_tools_amd/csrc/cc_host.hpp"

using namespace cc;

__global__ void k_read(const float4* __restrict__ in, int64_t n4, float* out) {
    float acc = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
        const float4 v = in[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 1234.5f) out[0] = acc;
}

__global__ void k_write(ulonglong2* __restrict__ out, int64_t n2) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = make_ulonglong2((u64)i, 0);
}

template <class F>
static double time_ms(hipStream_t s, int iters, F&& f) {
    hipEvent_t a, b;
    HIP_OK(hipEventCreate(&a));
    HIP_OK(hipEventCreate(&b));
    f();   // warm-up
    HIP_OK(hipGetLastError());
    HIP_OK(hipEventRecord(a, s));
    for (int i = 0; i < iters; ++i) f();
    HIP_OK(hipEventRecord(b, s));
    HIP_OK(hipEventSynchronize(b));
    HIP_OK(hipGetLastError());
    float ms = 0;
    HIP_OK(hipEventElapsedTime(&ms, a, b));
    HIP_OK(hipEventDestroy(a));
    HIP_OK(hipEventDestroy(b));
    return ms / iters;
}

int main(int argc, char** argv) {
    try {
        if (argc < 7) {
            std::fprintf(stderr, "usage: %s Z Y X bz by bx [mode] [iters]\n", argv[0]);
            return 2;
        }
        const int64_t shape[3] = {atoll(argv[1]), atoll(argv[2]), atoll(argv[3])};
        const int64_t bs[3] = {atoll(argv[4]), atoll(argv[5]), atoll(argv[6])};
        const int mode = argc > 7 ? atoi(argv[7]) : 0;
        const int iters = argc > 8 ? atoi(argv[8]) : 10;
        HostGeom hg = make_geom(shape, bs, 0);
        Geom& g = hg.g;
        const int64_t nt = g.n_tiles, nb = g.n_blocks, nvox = hg.nvox;
        const uint64_t nodes = (uint64_t)nt * g.cap;
        hipStream_t s;
        HIP_OK(hipStreamCreate(&s));
        int32_t* tab;
        HIP_OK(hipMalloc(&tab, hg.tab.size() * 4));
        HIP_OK(hipMemcpy(tab, hg.tab.data(), hg.tab.size() * 4, hipMemcpyHostToDevice));
        bind_geom_tables(hg, tab);
        float* in;
        u64* out;
        HIP_OK(hipMalloc(&in, nvox * 4));
        HIP_OK(hipMalloc(&out, nvox * 8));
        {
            const int64_t nxb = (shape[2] + 255) / 256;
            k_generate<<<dim3((unsigned)(shape[1] * nxb), (unsigned)shape[0]), 256, 0, s>>>(in, shape[0], shape[1], shape[2], 0, 0, 0, 0x5EED, 0);
        }
        u32 *st, *COUNT, *P;
        face_t* FACES;
        u64 *BITS, *KEY, *FIN;
        BlockParam* bp;
        float* dummy;
        HIP_OK(hipMalloc(&st, nb * 12));
        HIP_OK(hipMalloc(&bp, nb * sizeof(BlockParam)));
        HIP_OK(hipMalloc(&BITS, nt * NROWS * 8));
        HIP_OK(hipMalloc(&FACES, nt * FACE_STRIDE * 4));
        HIP_OK(hipMalloc(&COUNT, nt * 4));
        HIP_OK(hipMalloc(&P, nodes * 4));
        HIP_OK(hipMalloc(&KEY, nodes * 8));
        HIP_OK(hipMalloc(&FIN, nodes * 8));
        HIP_OK(hipMalloc(&dummy, 64));
        HIP_OK(hipMemset(FIN, 0, nodes * 8));
        u32 *smin = st, *smax = st + nb, *sflag = st + 2 * nb;
        const float thr = 0.5f;
        auto stats = [&] {
            HIP_OK(hipMemsetAsync(smin, 0xFF, nb * 4, s));
            HIP_OK(hipMemsetAsync(smax, 0, 2 * nb * 4, s));
            k_block_stats<<<(unsigned)nt, NTHREADS, 0, s>>>(g, in, smin, smax, sflag);
        };
        stats();
        k_block_params<<<(unsigned)((nb + 255) / 256), 256, 0, s>>>(nb, smin, smax, sflag, thr, mode, bp);
        HIP_OK(hipStreamSynchronize(s));

        std::vector<std::pair<const char*, double>> r;
        const unsigned big = 8 * 256 * 4;
        r.push_back({"copy_read", time_ms(s, iters, [&] { k_read<<<big, 256, 0, s>>>((const float4*)in, nvox / 4, dummy); })});
        r.push_back({"copy_write", time_ms(s, iters, [&] { k_write<<<big, 256, 0, s>>>((ulonglong2*)out, nvox / 2); })});
        r.push_back({"k_block_stats", time_ms(s, iters, stats)});
#define P1(A) k_pass1<false, A><<<(unsigned)nt, NTHREADS, 0, s>>>(g, in, nullptr, bp, thr, mode, BITS, FACES, COUNT, P, KEY)
        r.push_back({"k_pass1_abl1_load_bits", time_ms(s, iters, [&] { P1(1); })});
        r.push_back({"k_pass1_ccl_ph1_runs", time_ms(s, iters, [&] { P1(11); })});
        r.push_back({"k_pass1_ccl_ph2_unions", time_ms(s, iters, [&] { P1(12); })});
        r.push_back({"k_pass1_ccl_ph3_compress", time_ms(s, iters, [&] { P1(13); })});
        r.push_back({"k_pass1_abl2_ccl", time_ms(s, iters, [&] { P1(2); })});
        r.push_back({"k_pass1_abl3_keys", time_ms(s, iters, [&] { P1(3); })});
        r.push_back({"k_pass1_full", time_ms(s, iters, [&] { P1(0); })});
        // speculative front: sample + guess, k_spec with the exact parameters as the guess (no relabel)
        {
            u32 *fst, *part, *TB;
            BlockParam* guess;
            HIP_OK(hipMalloc(&fst, 3 * nb * 4));
            HIP_OK(hipMalloc(&part, nb * SAMPLE_PARTS * 16));
            HIP_OK(hipMalloc(&TB, nt * 16));
            HIP_OK(hipMalloc(&guess, nb * sizeof(BlockParam)));
            r.push_back({"k_sample_guess", time_ms(s, iters, [&] {
                k_sample<<<(unsigned)(nb * SAMPLE_PARTS), NTHREADS, 0, s>>>(g, in, part, FrontClear{});
                k_guess<<<(unsigned)((nb + 255) / 256), 256, 0, s>>>(nb, part, thr, mode, guess);
            })});
            std::vector<BlockParam> hb(nb);
            HIP_OK(hipMemcpy(hb.data(), bp, nb * sizeof(BlockParam), hipMemcpyDeviceToHost));
            for (auto& q : hb)
                if (q.kind == BP_INTERVAL) { if (mode == 0) q.hi = 0xFFFFFFFFu; else if (mode == 1) q.lo = 0; }
            HIP_OK(hipMemcpy(guess, hb.data(), nb * sizeof(BlockParam), hipMemcpyHostToDevice));
            SpecArgs sa;
            sa.guess = guess; sa.smin = fst; sa.smax = fst + nb; sa.sflag = fst + 2 * nb; sa.TB = TB; sa.t0 = 0;
            r.push_back({"k_spec", time_ms(s, iters, [&] {
                HIP_OK(hipMemsetAsync(fst, 0xFF, nb * 4, s));
                HIP_OK(hipMemsetAsync(fst + nb, 0, 2 * nb * 4, s));
                if (mode == 0) k_spec<false, 1><<<(unsigned)nt, NTHREADS, 0, s>>>(g, sa, in, nullptr, BITS, FACES, COUNT, P, KEY);
                else if (mode == 1) k_spec<false, 2><<<(unsigned)nt, NTHREADS, 0, s>>>(g, sa, in, nullptr, BITS, FACES, COUNT, P, KEY);
                else k_spec<false, 3><<<(unsigned)nt, NTHREADS, 0, s>>>(g, sa, in, nullptr, BITS, FACES, COUNT, P, KEY);
            })});
#define SPS(A) k_spec<false, 1, A><<<(unsigned)nt, NTHREADS, 0, s>>>(g, sa, in, nullptr, BITS, FACES, COUNT, P, KEY)
            r.push_back({"k_spec_nobits", time_ms(s, iters, [&] { SPS(20); })});
            r.push_back({"k_spec_nofaces", time_ms(s, iters, [&] { SPS(21); })});
            r.push_back({"k_spec_nostores", time_ms(s, iters, [&] { SPS(22); })});
            r.push_back({"k_spec_rows", time_ms(s, iters, [&] { SPS(99); })});
            r.push_back({"k_spec_bits", time_ms(s, iters, [&] { SPS(1); })});
            r.push_back({"k_spec_ph2", time_ms(s, iters, [&] { SPS(12); })});
            r.push_back({"k_spec_ccl", time_ms(s, iters, [&] { SPS(2); })});
            r.push_back({"k_spec_keys", time_ms(s, iters, [&] { SPS(3); })});
        }
        // compute-bound variants: every tile reads one of 8 tiles that stay in L2 (tile origins
        // z = y = 0, x = 64 (ix % 8)); outputs per tile as usual
        {
            std::vector<int32_t> tab2 = hg.tab;
            const int n0 = g.nt[0], n1 = g.nt[1], n2 = g.nt[2];
            for (int i = 0; i < n0; ++i) tab2[i] = 0;
            for (int i = 0; i < n1; ++i) tab2[3 * n0 + i] = 0;
            for (int i = 0; i < n2; ++i) tab2[3 * n0 + 3 * n1 + i] = (i % 8) * 64;
            int32_t* tabc;
            HIP_OK(hipMalloc(&tabc, tab2.size() * 4));
            HIP_OK(hipMemcpy(tabc, tab2.data(), tab2.size() * 4, hipMemcpyHostToDevice));
            HostGeom hc = hg;
            bind_geom_tables(hc, tabc);
            Geom gc = hc.g;
            u32 *fst, *TB;
            BlockParam* guess;
            HIP_OK(hipMalloc(&fst, 3 * nb * 4));
            HIP_OK(hipMalloc(&TB, nt * 16));
            HIP_OK(hipMalloc(&guess, nb * sizeof(BlockParam)));
            HIP_OK(hipMemcpy(guess, bp, nb * sizeof(BlockParam), hipMemcpyDeviceToDevice));
            SpecArgs sa;
            sa.guess = guess; sa.smin = fst; sa.smax = fst + nb; sa.sflag = fst + 2 * nb; sa.TB = TB; sa.t0 = 0;
            r.push_back({"k_spec_cached", time_ms(s, iters, [&] {
                k_spec<false, 1><<<(unsigned)nt, NTHREADS, 0, s>>>(gc, sa, in, nullptr, BITS, FACES, COUNT, P, KEY);
            })});
#define SPC(A) k_spec<false, 1, A><<<(unsigned)nt, NTHREADS, 0, s>>>(gc, sa, in, nullptr, BITS, FACES, COUNT, P, KEY)
            r.push_back({"k_spec_rows_cached", time_ms(s, iters, [&] { SPC(99); })});
            r.push_back({"k_spec_bits_cached", time_ms(s, iters, [&] { SPC(1); })});
            r.push_back({"k_spec_ph1_cached", time_ms(s, iters, [&] { SPC(11); })});
            r.push_back({"k_spec_ph2_cached", time_ms(s, iters, [&] { SPC(12); })});
            r.push_back({"k_spec_ph3_cached", time_ms(s, iters, [&] { SPC(13); })});
            r.push_back({"k_spec_ccl_cached", time_ms(s, iters, [&] { SPC(2); })});
            r.push_back({"k_spec_keys_cached", time_ms(s, iters, [&] { SPC(3); })});
            r.push_back({"k_block_stats_cached", time_ms(s, iters, [&] {
                k_block_stats<<<(unsigned)nt, NTHREADS, 0, s>>>(gc, in, smin, smax, sflag);
            })});
#define P1C(A) k_pass1<false, A><<<(unsigned)nt, NTHREADS, 0, s>>>(gc, in, nullptr, bp, thr, mode, BITS, FACES, COUNT, P, KEY)
            r.push_back({"k_pass1_abl1_cached", time_ms(s, iters, [&] { P1C(1); })});
            r.push_back({"k_pass1_ph1_cached", time_ms(s, iters, [&] { P1C(11); })});
            r.push_back({"k_pass1_ph2list_cached", time_ms(s, iters, [&] { P1C(14); })});
            r.push_back({"k_pass1_ph2_cached", time_ms(s, iters, [&] { P1C(12); })});
            r.push_back({"k_pass1_ph3_cached", time_ms(s, iters, [&] { P1C(13); })});
            r.push_back({"k_pass1_abl2_cached", time_ms(s, iters, [&] { P1C(2); })});
            r.push_back({"k_pass1_abl3_cached", time_ms(s, iters, [&] { P1C(3); })});
            r.push_back({"k_pass1_full_cached", time_ms(s, iters, [&] { P1C(0); })});
        }
        // seam kernel variants (FACES from the last full pass-1 run above)
        {
            P1(0);
            u64 *pairs, *ipairs;
            u32 *pc, *ipc;
            u8 *big, *iovf;
            HIP_OK(hipMalloc(&pairs, (size_t)nt * TPC * 8));
            HIP_OK(hipMalloc(&ipairs, (size_t)nt * TPI * 8));
            HIP_OK(hipMalloc(&pc, nt * 4));
            HIP_OK(hipMalloc(&ipc, nt * 4));
            HIP_OK(hipMalloc(&big, nb));
            HIP_OK(hipMalloc(&iovf, nt));
            HIP_OK(hipMemset(big, 0, nb));
            HIP_OK(hipMemset(iovf, 0, nt));
            const unsigned sg = (unsigned)((nt + SP_WAVES - 1) / SP_WAVES);
#define SEAMS(V) k_seams<V><<<sg, SP_WAVES * 64, 0, s>>>(g, FACES, COUNT, pairs, pc, big, ipairs, ipc, iovf, 0, nt, nullptr)
            r.push_back({"k_seams_stage", time_ms(s, iters, [&] { SEAMS(1); })});
            r.push_back({"k_seams_z", time_ms(s, iters, [&] { SEAMS(2); })});
            r.push_back({"k_seams_zy", time_ms(s, iters, [&] { SEAMS(3); })});
            r.push_back({"k_seams_zyx", time_ms(s, iters, [&] { SEAMS(4); })});
            r.push_back({"k_seams_full", time_ms(s, iters, [&] { SEAMS(0); })});
        }
        r.push_back({"k_pass2", time_ms(s, iters, [&] { k_pass2<false><<<(unsigned)nt, NTHREADS, 0, s>>>(g, BITS, COUNT, FIN, nullptr, nullptr, 0, 0, out, 0, nullptr, nullptr); })});
        std::printf("{\"shape\": [%lld, %lld, %lld], \"block\": [%lld, %lld, %lld], \"mode\": %d, \"tiles\": %lld",
                    (long long)shape[0], (long long)shape[1], (long long)shape[2], (long long)bs[0], (long long)bs[1],
                    (long long)bs[2], mode, (long long)nt);
        for (auto& kv : r) std::printf(", \"%s\": %.4f", kv.first, kv.second);
        std::printf("}\n");
        auto ms = [&](const char* name) {
            for (auto& kv : r) if (std::string(kv.first) == name) return kv.second;
            return 0.0;
        };
        std::printf("# GB/s: read %.0f  write %.0f  stats %.0f  k_spec(4B/vox) %.0f  pass2(8B/vox) %.0f\n",
                    nvox * 4 / ms("copy_read") / 1e6, nvox * 8 / ms("copy_write") / 1e6, nvox * 4 / ms("k_block_stats") / 1e6,
                    nvox * 4 / ms("k_spec") / 1e6, nvox * 8 / ms("k_pass2") / 1e6);
    } catch (const CCError& e) {
        std::fprintf(stderr, "error: %s\n", e.msg.c_str());
        return 1;
    }
    return 0;
}
