// tools/spec_check.hip -- development check of the speculative front (not part of the library):
// k_spec with the exact block parameters as its guess must reproduce k_pass1's bit rows and
// counts; prints the k_sample guesses beside the exact parameters.
// Build: make -C tools spec_check   Run: tools/spec_check Z Y X bz by bx [mode]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../cluster_tools_amd/csrc/cc_kernels.hip"
#include "../cluster_tools_amd/csrc/cc_generate.hip"
#include "../cluster_tools_amd/csrc/cc_host.hpp"

using namespace cc;

int main(int argc, char** argv) {
    try {
        if (argc < 7) return 2;
        const int64_t shape[3] = {atoll(argv[1]), atoll(argv[2]), atoll(argv[3])};
        const int64_t bs[3] = {atoll(argv[4]), atoll(argv[5]), atoll(argv[6])};
        const int mode = argc > 7 ? atoi(argv[7]) : 0;
        HostGeom hg = make_geom(shape, bs, 0);
        Geom& g = hg.g;
        const int64_t nt = g.n_tiles, nb = g.n_blocks, nvox = hg.nvox;
        const uint64_t nodes = (uint64_t)nt * g.cap;
        hipStream_t s = 0;
        int32_t* tab;
        HIP_OK(hipMalloc(&tab, hg.tab.size() * 4));
        HIP_OK(hipMemcpy(tab, hg.tab.data(), hg.tab.size() * 4, hipMemcpyHostToDevice));
        bind_geom_tables(hg, tab);
        float* in;
        HIP_OK(hipMalloc(&in, nvox * 4));
        {
            const int64_t nxb = (shape[2] + 255) / 256;
            k_generate<<<dim3((unsigned)(shape[1] * nxb), (unsigned)shape[0]), 256, 0, s>>>(in, shape[0], shape[1], shape[2], 0, 0, 0, 0x5EED, 0);
        }
        u32 *st, *COUNT[2], *P, *TB;
        face_t* FACES;
        u64 *BITS[2], *KEY;
        BlockParam *bp, *guess;
        HIP_OK(hipMalloc(&st, nb * 12));
        HIP_OK(hipMalloc(&bp, nb * sizeof(BlockParam)));
        HIP_OK(hipMalloc(&guess, nb * sizeof(BlockParam)));
        for (int i = 0; i < 2; ++i) {
            HIP_OK(hipMalloc(&BITS[i], nt * NROWS * 8));
            HIP_OK(hipMalloc(&COUNT[i], nt * 4));
        }
        HIP_OK(hipMalloc(&FACES, nt * FACE_STRIDE * 4));
        HIP_OK(hipMalloc(&P, nodes * 4));
        HIP_OK(hipMalloc(&KEY, nodes * 8));
        HIP_OK(hipMalloc(&TB, nt * 16));
        u32 *smin = st, *smax = st + nb, *sflag = st + 2 * nb;
        const float thr = 0.5f;
        HIP_OK(hipMemset(smin, 0xFF, nb * 4));
        HIP_OK(hipMemset(smax, 0, 2 * nb * 4));
        k_block_stats<<<(unsigned)nt, NTHREADS, 0, s>>>(g, in, smin, smax, sflag);
        k_block_params<<<(unsigned)((nb + 255) / 256), 256, 0, s>>>(nb, smin, smax, sflag, thr, mode, bp);
        k_pass1<false, 0><<<(unsigned)nt, NTHREADS, 0, s>>>(g, in, nullptr, bp, thr, mode, BITS[0], FACES, COUNT[0], P, KEY);
        u32* part;
        HIP_OK(hipMalloc(&part, nb * SAMPLE_PARTS * 16));
        k_sample<<<(unsigned)(nb * SAMPLE_PARTS), NTHREADS, 0, s>>>(g, in, part, FrontClear{});
        k_guess<<<(unsigned)((nb + 255) / 256), 256, 0, s>>>(nb, part, thr, mode, guess);
        HIP_OK(hipDeviceSynchronize());
        std::vector<BlockParam> hb(nb), hgs(nb);
        HIP_OK(hipMemcpy(hb.data(), bp, nb * sizeof(BlockParam), hipMemcpyDeviceToHost));
        HIP_OK(hipMemcpy(hgs.data(), guess, nb * sizeof(BlockParam), hipMemcpyDeviceToHost));
        for (int64_t b = 0; b < nb && b < 8; ++b)
            std::printf("block %ld exact kind %u lo %08x hi %08x | guess kind %u lo %08x hi %08x\n", (long)b, hb[b].kind,
                        hb[b].lo, hb[b].hi, hgs[b].kind, hgs[b].lo, hgs[b].hi);
        // guess := exact (widened)
        for (auto& p : hb) {
            if (p.kind == BP_INTERVAL) { if (mode == 0) p.hi = 0xFFFFFFFFu; else if (mode == 1) p.lo = 0; }
        }
        HIP_OK(hipMemcpy(guess, hb.data(), nb * sizeof(BlockParam), hipMemcpyHostToDevice));
        SpecArgs sa;
        sa.guess = guess; sa.smin = smin; sa.smax = smax; sa.sflag = sflag; sa.TB = TB; sa.t0 = 0;
        if (mode == 0) k_spec<false, 1><<<(unsigned)nt, NTHREADS, 0, s>>>(g, sa, in, nullptr, BITS[1], FACES, COUNT[1], P, KEY);
        else if (mode == 1) k_spec<false, 2><<<(unsigned)nt, NTHREADS, 0, s>>>(g, sa, in, nullptr, BITS[1], FACES, COUNT[1], P, KEY);
        else k_spec<false, 3><<<(unsigned)nt, NTHREADS, 0, s>>>(g, sa, in, nullptr, BITS[1], FACES, COUNT[1], P, KEY);
        HIP_OK(hipDeviceSynchronize());
        std::vector<u64> b0(nt * NROWS), b1(nt * NROWS);
        std::vector<u32> c0(nt), c1(nt);
        HIP_OK(hipMemcpy(b0.data(), BITS[0], nt * NROWS * 8, hipMemcpyDeviceToHost));
        HIP_OK(hipMemcpy(b1.data(), BITS[1], nt * NROWS * 8, hipMemcpyDeviceToHost));
        HIP_OK(hipMemcpy(c0.data(), COUNT[0], nt * 4, hipMemcpyDeviceToHost));
        HIP_OK(hipMemcpy(c1.data(), COUNT[1], nt * 4, hipMemcpyDeviceToHost));
        int64_t bad = 0, badc = 0;
        for (int64_t i = 0; i < nt * NROWS; ++i)
            if (b0[i] != b1[i]) {
                if (bad < 8) std::printf("row %ld (tile %ld row %ld): pass1 %016lx spec %016lx\n", (long)i, (long)(i / NROWS),
                                         (long)(i % NROWS), (unsigned long)b0[i], (unsigned long)b1[i]);
                ++bad;
            }
        for (int64_t t = 0; t < nt; ++t) badc += c0[t] != c1[t];
        std::printf("rows differing %ld / %ld, counts differing %ld / %ld\n", (long)bad, (long)(nt * NROWS), (long)badc, (long)nt);
        return bad || badc ? 1 : 0;
    } catch (const CCError& e) {
        std::fprintf(stderr, "error: %s\n", e.msg.c_str());
        return 1;
    }
}
