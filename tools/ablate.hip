// tools/ablate.hip -- kernel ablation / roofline harness (timing only, not part of the library).
//
// Runs the volume-sized kernels of the path on a synthetic boundary map already in HBM and times
// each variant with HIP events over `iters` launches:
//   copy_read / copy_write   plain float4 streaming read / 16-B uint64 store (the box's HBM ceiling)
//   k_block_stats            per-block min/max pass
//   k_pass1 ABL=1,2,3,0      stop after: load+threshold+bits | + tile CCL | + first voxels | full
//   k_front lag 1..3         stats + params + pass 1 fused, Infinity-Cache ordered
//   k_pass2                  relabel + uint64 write (FIN = 0: timing only)
// Build: make -C tools ablate   Run: tools/ablate Z Y X bz by bx [mode] [iters]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
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

// stats in block-major tile order (one workgroup per tile); interleave > 1: only every
// interleave-th workgroup works, in runs of per_block (the others exit at once)
__global__ __launch_bounds__(NTHREADS) void k_stats_bm(Geom g, const float* __restrict__ in, u32* smin, u32* smax,
                                                       u32* sflag, int per_block, int interleave) {
    __shared__ u32 red[3][NTHREADS / 64];
    extern __shared__ u32 dyn[];
    int64_t idx = blockIdx.x;
    if (interleave > 1) {
        const int64_t run = idx / per_block;
        if (run % interleave) return;
        idx = (run / interleave) * per_block + idx % per_block;
    }
    if (dyn[0] == 0x12345678u) return;
    const int64_t b = idx / per_block;
    const int64_t t = block_tile(g, b, (int)(idx % per_block));
    stats_tile(g, tile_info(g, t), in, smin, smax, sflag, red);
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
            k_generate<<<dim3((unsigned)(shape[1] * nxb), (unsigned)shape[0]), 256, 0, s>>>(in, shape[0], shape[1], shape[2], 0, 0, 0, 0x5EED);
        }
        u32 *st, *COUNT, *P, *FACES;
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
        if (nt % nb == 0)
        {
            r.push_back({"k_stats_blockmajor", time_ms(s, iters, [&] {
                k_stats_bm<<<(unsigned)nt, NTHREADS, 16, s>>>(g, in, smin, smax, sflag, (int)(nt / nb), 1); })});
            r.push_back({"k_stats_bm_lds38k_unused", time_ms(s, iters, [&] {
                k_stats_bm<<<(unsigned)nt, NTHREADS, 38400, s>>>(g, in, smin, smax, sflag, (int)(nt / nb), 1); })});
            r.push_back({"k_stats_bm_interleave2", time_ms(s, iters, [&] {
                k_stats_bm<<<(unsigned)(2 * nt), NTHREADS, 16, s>>>(g, in, smin, smax, sflag, (int)(nt / nb), 2); })});
            r.push_back({"k_stats_bm_interleave2_lds38k", time_ms(s, iters, [&] {
                k_stats_bm<<<(unsigned)(2 * nt), NTHREADS, 38400, s>>>(g, in, smin, smax, sflag, (int)(nt / nb), 2); })});
        }
#define P1(A) k_pass1<false, A><<<(unsigned)nt, NTHREADS, 0, s>>>(g, in, nullptr, bp, thr, mode, BITS, FACES, COUNT, P, KEY)
        r.push_back({"k_pass1_abl1_load_bits", time_ms(s, iters, [&] { P1(1); })});
        r.push_back({"k_pass1_ccl_ph1_runs", time_ms(s, iters, [&] { P1(11); })});
        r.push_back({"k_pass1_ccl_ph2_unions", time_ms(s, iters, [&] { P1(12); })});
        r.push_back({"k_pass1_ccl_ph3_compress", time_ms(s, iters, [&] { P1(13); })});
        r.push_back({"k_pass1_abl2_ccl", time_ms(s, iters, [&] { P1(2); })});
        r.push_back({"k_pass1_abl3_keys", time_ms(s, iters, [&] { P1(3); })});
        r.push_back({"k_pass1_full", time_ms(s, iters, [&] { P1(0); })});
        // fused front (stats + params + pass 1 in one launch)
        {
            u32* fst;
            int64_t* fseg;
            u64* items;
            HIP_OK(hipMalloc(&fst, (5 * nb + 2) * 4));
            HIP_OK(hipMalloc(&fseg, (4 * nb + 4) * 8));
            HIP_OK(hipMalloc(&items, 2 * nt * 8));
            std::vector<int64_t> hseg;
            static const char* fnames[10] = {"k_front_lag1", "k_front_lag2", "k_front_lag1_nowait", "k_front_stats_only",
                                            "k_front_pass1_only", "k_front_ticket_only", "k_front_lag1_s2",
                                            "k_front_lag1_s3", "k_front_lag1_s4", "k_front_lag2_s2"};
            for (int v = 0; v < 10; ++v) {
                const int lag = v == 1 || v == 9 ? 2 : 1;
                const int per_s = v == 6 || v == 9 ? 2 : v == 7 ? 3 : v == 8 ? 4 : 1, per_p = 1;
                const int64_t nseg = build_front_segments(hg, lag, hseg, per_s, per_p);
                const int64_t n_items = hseg[nseg];
                HIP_OK(hipMemcpy(fseg, hseg.data(), hseg.size() * 8, hipMemcpyHostToDevice));
                k_front_items<<<1024, 256, 0, s>>>(g, fseg, (int32_t)nseg, per_s, per_p, items);
                FrontArgs fa;
                fa.items = items; fa.n_items = n_items; fa.per_s = per_s; fa.per_p = per_p;
                fa.smin = fst; fa.smax = fst + nb; fa.sflag = fst + 2 * nb; fa.sdone = fst + 3 * nb; fa.ready = fst + 4 * nb;
                fa.bp = bp; fa.queue = fst + 5 * nb;
                r.push_back({fnames[v], time_ms(s, iters, [&] {
                    HIP_OK(hipMemsetAsync(fst, 0xFF, nb * 4, s));
                    HIP_OK(hipMemsetAsync(fst + nb, 0, (4 * nb + 2) * 4, s));
                    const unsigned grid = (unsigned)n_items;
                    const int tv = v < 2 || v >= 6 ? 0 : v == 2 ? 2 : v == 3 ? 3 : v == 4 ? 4 : 6;
                    if (tv == 0) k_front<0><<<grid, NTHREADS, 0, s>>>(g, fa, in, thr, mode, BITS, FACES, COUNT, P, KEY);
                    else if (tv == 2) k_front<2><<<grid, NTHREADS, 0, s>>>(g, fa, in, thr, mode, BITS, FACES, COUNT, P, KEY);
                    else if (tv == 3) k_front<3><<<grid, NTHREADS, 0, s>>>(g, fa, in, thr, mode, BITS, FACES, COUNT, P, KEY);
                    else if (tv == 4) k_front<4><<<grid, NTHREADS, 0, s>>>(g, fa, in, thr, mode, BITS, FACES, COUNT, P, KEY);
                    else k_front<6><<<grid, NTHREADS, 0, s>>>(g, fa, in, thr, mode, BITS, FACES, COUNT, P, KEY);
                })});
                u32 err = 0;
                HIP_OK(hipMemcpy(&err, fst + 5 * nb + 1, 4, hipMemcpyDeviceToHost));
                if (err) std::fprintf(stderr, "k_front variant %d: wait timeout flagged\n", v);
            }
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
#define SEAMS(V) k_seams<V><<<sg, SP_WAVES * 64, 0, s>>>(g, FACES, pairs, pc, big, ipairs, ipc, iovf)
            r.push_back({"k_seams_stage", time_ms(s, iters, [&] { SEAMS(1); })});
            r.push_back({"k_seams_z", time_ms(s, iters, [&] { SEAMS(2); })});
            r.push_back({"k_seams_zy", time_ms(s, iters, [&] { SEAMS(3); })});
            r.push_back({"k_seams_zyx", time_ms(s, iters, [&] { SEAMS(4); })});
            r.push_back({"k_seams_full", time_ms(s, iters, [&] { SEAMS(0); })});
        }
        r.push_back({"k_pass2", time_ms(s, iters, [&] { k_pass2<<<(unsigned)nt, NTHREADS, 0, s>>>(g, BITS, COUNT, FIN, out); })});
        std::printf("{\"shape\": [%lld, %lld, %lld], \"block\": [%lld, %lld, %lld], \"mode\": %d, \"tiles\": %lld",
                    (long long)shape[0], (long long)shape[1], (long long)shape[2], (long long)bs[0], (long long)bs[1],
                    (long long)bs[2], mode, (long long)nt);
        for (auto& kv : r) std::printf(", \"%s\": %.4f", kv.first, kv.second);
        std::printf("}\n");
        std::printf("# GB/s: read %.0f  write %.0f  stats %.0f  pass1(4B/vox) %.0f  pass2(8B/vox) %.0f\n",
                    nvox * 4 / r[0].second / 1e6, nvox * 8 / r[1].second / 1e6, nvox * 4 / r[2].second / 1e6,
                    nvox * 4 / r[10].second / 1e6, nvox * 8 / r.back().second / 1e6);
    } catch (const CCError& e) {
        std::fprintf(stderr, "error: %s\n", e.msg.c_str());
        return 1;
    }
    return 0;
}
