// cc_rows.hpp -- device helpers shared by both translation units of the library (cc_lib.hip:
// the labelling path; cc_aux.hip: evaluation, relabelling, prefilter, watershed): the
// coalesced walk over a tile's voxel rows and the per-block statistics built on it.
#pragma once
#include "cc_common.hpp"

namespace cc {

// ------------------------------------------------------------------------------------------
// k_block_stats: per-block ordered min / max and NaN flag.  One workgroup per tile, lane = x.
// ------------------------------------------------------------------------------------------
// Visit every voxel row of the tile, lane = x: f(j, value, mask byte) for the wave's rows
// (lz, ly = wave + NW * b), j = lz * RY + b in [0, TZ * RY) the row's slot in the wave (a
// compile-time constant: the loops are fully unrolled).  One 4-B
// load per lane and row (256 B per wave instruction) from SGPR row pointers; RZ planes x RY rows
// = 16 loads in flight per wave.  Full tiles take a branch-free path; on edge tiles lanes past the
// x extent re-load the last column (duplicates: harmless to min / max; the bit rows are masked
// by the caller) and rows past the extent are skipped (f is not called for them).
constexpr int RZ = 4;                       // planes per round
// the input's loads (CC_ROWS_NT, A/B only: non-temporal, as k_spec's float4 path -- C1 k_spec 0.258
// -> 0.223 ms but k_pass2 0.433 -> 0.484 ms after it, profiles/r05_ab_ntload.txt)
#ifndef CC_ROWS_NT
#define CC_ROWS_NT 0
#endif
__device__ __forceinline__ float ld_row(const float* p) {
    if constexpr (CC_ROWS_NT) return __builtin_nontemporal_load(p);
    else return *p;
}
#ifndef CC_MASK_RZ
#define CC_MASK_RZ 2
#endif
constexpr int NWAVE = NTHREADS / 64;
constexpr int RY = TY / NWAVE;              // rows per plane and wave
static_assert(TZ * RY == 64, "one wave slot per row: a wave owns 64 rows of a tile");

__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(cc_tid() >> 6); }

template <bool HAS_MASK, class F>
__device__ __forceinline__ void for_tile_rows(const Geom& g, const TileInfo& ti, const float* __restrict__ in,
                                              const u8* __restrict__ mask, F&& f) {
    const int lane = cc_tid() & 63, wave = wave_id();
    // planes per round: RZ, or 2 with a mask (its bytes in flight too; RZ = 4 spilled)
    constexpr int RZ_ = HAS_MASK ? CC_MASK_RZ : RZ;
    const int64_t sz = g.Y * g.X, sy = NWAVE * g.X;
    const int64_t o0 = ((int64_t)ti.z0 * g.Y + ti.y0 + wave) * g.X + ti.x0;
    if (ti.lz == TZ && ti.ly == TY && ti.lx == TX) {
        const float* pz = in + o0;
        const u8* mz = HAS_MASK ? mask + o0 : nullptr;
#pragma unroll
        for (int z0 = 0; z0 < TZ; z0 += RZ_, pz += RZ_ * sz) {
            float v[RZ_][RY];
            u8 mk[RZ_][RY];
#pragma unroll
            for (int a = 0; a < RZ_; ++a)
#pragma unroll
                for (int b = 0; b < RY; ++b) {
                    v[a][b] = ld_row(pz + a * sz + b * sy + lane);
                    if (HAS_MASK) mk[a][b] = mz[(z0 + a) * sz + b * sy + lane];
                }
#pragma unroll
            for (int a = 0; a < RZ_; ++a)
#pragma unroll
                for (int b = 0; b < RY; ++b) f((z0 + a) * RY + b, v[a][b], HAS_MASK ? (u32)mk[a][b] : 1u);
        }
        return;
    }
    const int lx = lane < ti.lx ? lane : ti.lx - 1;
#pragma unroll
    for (int z0 = 0; z0 < TZ; z0 += RZ_) {
        if (z0 >= ti.lz) break;
        float v[RZ_][RY];
        u8 mk[RZ_][RY];
#pragma unroll
        for (int a = 0; a < RZ_; ++a)
#pragma unroll
            for (int b = 0; b < RY; ++b) {
                const int lz = z0 + a, ly = wave + NWAVE * b;
                v[a][b] = 0.0f;
                mk[a][b] = 0;
                if (lz < ti.lz && ly < ti.ly) {
                    const int64_t row = o0 + lz * sz + b * sy;
                    v[a][b] = ld_row(in + row + lx);
                    if (HAS_MASK) mk[a][b] = mask[row + lx];
                }
            }
#pragma unroll
        for (int a = 0; a < RZ_; ++a)
#pragma unroll
            for (int b = 0; b < RY; ++b) {
                const int lz = z0 + a, ly = wave + NWAVE * b;
                if (lz < ti.lz && ly < ti.ly) f(lz * RY + b, v[a][b], (u32)mk[a][b]);
            }
    }
}

// tile row index of wave slot j (see for_tile_rows)
__device__ __forceinline__ int slot_row(int j, int wave) { return (j / RY) * TY + wave + NWAVE * (j % RY); }

// ------------------------------------------------------------------------------------------
// k_block_stats: per-block ordered min / max and NaN flag.  One workgroup per tile.
// ------------------------------------------------------------------------------------------
// Stats of one tile folded into its block's (smin, smax, sflag); red = LDS scratch [3][WAVES].
__device__ __forceinline__ void stats_tile(const Geom& g, const TileInfo& ti, const float* __restrict__ in,
                                           u32* smin, u32* smax, u32* sflag, u32 (*red)[NTHREADS / 64]) {
    const int tid_ = cc_tid(), lane = tid_ & 63, wave = tid_ >> 6;
    u32 mn = 0xFFFFFFFFu, mx = 0u;
    // ordered min / max over all values; a NaN orders above +inf or below -inf, so the NaN flag
    // is read off the extremes instead of being tested per voxel
    for_tile_rows<false>(g, ti, in, nullptr, [&](int, float x, u32) {
        const u32 o = f2ord(__float_as_uint(x));
        mn = o < mn ? o : mn;
        mx = o > mx ? o : mx;
    });
    mn = wave_min(mn);
    mx = wave_max(mx);
    const bool anynan = mx > 0xFF800000u || mn < 0x007FFFFFu;      // > ord(+inf) or < ord(-inf)
    if (lane == 0) { red[0][wave] = mn; red[1][wave] = mx; red[2][wave] = anynan; }
    __syncthreads();
    if (tid_ == 0) {
        u32 a = red[0][0], b = red[1][0], f = red[2][0];
        for (int w = 1; w < NTHREADS / 64; ++w) {
            a = red[0][w] < a ? red[0][w] : a;
            b = red[1][w] > b ? red[1][w] : b;
            f |= red[2][w];
        }
        // returning atomics: the caller waits for them before it hands the block on
        const u32 o1 = atomicMin(smin + ti.block, a);
        const u32 o2 = atomicMax(smax + ti.block, b);
        const u32 o3 = f ? atomicOr(sflag + ti.block, 1u) : 0u;
        (void)o1; (void)o2; (void)o3;
    }
}

}  // namespace cc
