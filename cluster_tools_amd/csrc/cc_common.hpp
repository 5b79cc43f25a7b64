// cc_common.hpp -- shared device helpers for the MI355X thresholded-CCL library.
//
// Layout vocabulary:
//   block  = reference block of the block grid (nifty.tools.blocking, C-order ids,
//            cluster_tools/utils/volume_utils.py:31-77); normalisation and 26-connectivity
//            are per block, block faces stitch with 6-connectivity.
//   tile   = the unit one workgroup labels in LDS: TZ x TY x TX voxels, tiled from each
//            block's origin (so no tile straddles a block), truncated at block ends.
//   cube   = 2x2x2 voxels inside a tile (tile origin aligned); every foreground voxel of a
//            cube is 26-adjacent to every other, so a cube is one union-find node in LDS.
//   node   = a tile-local component; global id t*cap + k (k = its compact index in tile t).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace cc {

typedef uint64_t u64;
typedef uint32_t u32;
typedef uint8_t u8;

// Tile geometry.  TX = 64 so one tile row is one 64-bit ballot.
constexpr int TZ = 16, TY = 32, TX = 64;
constexpr int CZ = TZ / 2, CY = TY / 2, CX = TX / 2;
constexpr int NC = CZ * CY * CX;           // cubes per full tile (4096)
constexpr int NROWS = TZ * TY;             // bit rows per tile (512)
constexpr int NTHREADS = 512;              // 8 waves of 64
// face planes of a tile, in cubes; 16-bit entry = k | (4 face-voxel bits << FK_BITS), 0 = no
// face voxel (k < 4096: at most one component per cube)
constexpr int F_Z = CY * CX, F_Y = CZ * CX, F_X = CZ * CY;
constexpr int F_ZLO = 0, F_ZHI = F_Z, F_YLO = 2 * F_Z, F_YHI = 2 * F_Z + F_Y;
constexpr int F_XLO = 2 * F_Z + 2 * F_Y, F_XHI = 2 * F_Z + 2 * F_Y + F_X;
constexpr int FACE_STRIDE = 2 * (F_Z + F_Y + F_X);
using face_t = uint16_t;
constexpr int FK_BITS = 12;
constexpr unsigned FK_MASK = (1u << FK_BITS) - 1;
constexpr u32 NONE = 0xFFFFFFFFu;
constexpr int KEY_BITS = 36;               // packed sort key: block << 36 | first-voxel index

enum { MODE_GREATER = 0, MODE_LESS = 1, MODE_EQUAL = 2 };
enum { BP_EMPTY = 0, BP_INTERVAL = 1, BP_EXACT = 2 };

struct BlockParam {      // per reference block, from its min/max (volume_utils.py:98-105)
    float mn, m;         // min and max(x - min) (NaN where numpy's would be NaN)
    u32 lo, hi;          // foreground <=> lo <= ord(x) <= hi   (kind == BP_INTERVAL)
    u32 kind;
    u32 pad;
};

// block parameters read from global memory come back in VGPRs (the compiler cannot prove the
// buffer unwritten); branches on them must be seen as uniform or the writelane row collection in
// load_rows runs under a divergent region and produces wrong rows: move them to SGPRs
__device__ __forceinline__ BlockParam uniform_bp(const BlockParam& q) {
    BlockParam p;
    p.mn = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(q.mn)));
    p.m = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(q.m)));
    p.lo = __builtin_amdgcn_readfirstlane(q.lo);
    p.hi = __builtin_amdgcn_readfirstlane(q.hi);
    p.kind = __builtin_amdgcn_readfirstlane(q.kind);
    p.pad = 0;
    return p;
}

struct Geom {
    int64_t Z, Y, X;          // volume (or z-slab) shape
    int64_t zoff;             // global z of this volume's first plane (keys / multi-GPU)
    int64_t gY, gX;           // global Y, X (== Y, X)
    int32_t nb[3];            // blocks per axis
    int32_t nt[3];            // tiles per axis
    int64_t n_tiles;
    int64_t n_blocks;
    int32_t cap;              // node slots per tile (max cubes of any tile)
    int32_t pad;
    const int32_t* tstart[3]; // per-axis tile tables
    const int32_t* tlen[3];
    const int32_t* tblk[3];
    const int32_t* bt0[3];    // per-axis block tables: first tile index and tile count of a block
    const int32_t* btn[3];
};

struct TileInfo {
    int iz, iy, ix;
    int z0, y0, x0;
    int lz, ly, lx;
    int64_t block;
};

// thread index inside a 512-thread tile team (k_front runs two teams per workgroup)
__device__ __forceinline__ int cc_tid() { return threadIdx.x & (NTHREADS - 1); }

// tile ids fit u32 (node ids t * cap are u32, checked on the host): 32-bit division only
__device__ __forceinline__ TileInfo tile_info(const Geom& g, int64_t t) {
    TileInfo ti;
    const u32 tt = (u32)t, n2 = (u32)g.nt[2], n1 = (u32)g.nt[1];
    const u32 q = tt / n2, qz = q / n1;
    ti.ix = (int)(tt - q * n2);
    ti.iy = (int)(q - qz * n1);
    ti.iz = (int)qz;
    ti.z0 = g.tstart[0][ti.iz]; ti.lz = g.tlen[0][ti.iz];
    ti.y0 = g.tstart[1][ti.iy]; ti.ly = g.tlen[1][ti.iy];
    ti.x0 = g.tstart[2][ti.ix]; ti.lx = g.tlen[2][ti.ix];
    ti.block = ((int64_t)g.tblk[0][ti.iz] * g.nb[1] + g.tblk[1][ti.iy]) * g.nb[2] + g.tblk[2][ti.ix];
    return ti;
}

// IEEE-754 total order for non-NaN floats as unsigned ints (-0 < +0).
// (written as one xor with a sign-derived mask: v_ashrrev + v_bitop3 on gfx950, where the select
// form took four VALU ops per voxel)
__device__ __host__ __forceinline__ u32 f2ord(u32 u) { return u ^ ((u32)((int32_t)u >> 31) | 0x80000000u); }
__device__ __host__ __forceinline__ u32 ord2f(u32 o) { return (o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o; }

// The reference's per-voxel predicate with block statistics (block_components.py:161,166-173).
__device__ __forceinline__ bool exact_pred(float x, float mn, float m, float thr, int mode) {
    float y = x - mn;
    if (m > 0.0f) y = y / m;
    return mode == MODE_GREATER ? (y > thr) : mode == MODE_LESS ? (y < thr) : (y == thr);
}

__device__ __forceinline__ bool voxel_pred(const BlockParam& p, float x, float thr, int mode) {
    if (p.kind == BP_INTERVAL) {
        u32 o = f2ord(__float_as_uint(x));
        return o >= p.lo && o <= p.hi;
    }
    if (p.kind == BP_EXACT) return exact_pred(x, p.mn, p.m, thr, mode);
    return false;
}

// ---- LDS union-find over cubes (root = smallest cube index of the component) ----
// LDS pointers with an explicit address space: volatile accesses through a generic pointer
// are not narrowed to LDS by the compiler and would become flat_load / flat_store.
typedef __attribute__((address_space(3))) u32 lds_u32;
__device__ __forceinline__ lds_u32* as_lds(u32* p) { return (lds_u32*)p; }

// find with path halving.  Only ever stores an ancestor of x into par[x] (same set,
// smaller index), which keeps the concurrent atomicMin-based unions correct.
__device__ __forceinline__ u32 lfind(volatile lds_u32* par, u32 x) {
    u32 p = par[x];
    while (p != x) {
        const u32 gp = par[p];
        if (gp == p) return p;
        par[x] = gp;
        x = gp;
        p = par[x];
    }
    return x;
}

// root of x without path compression (concurrent stores of ancestors by other threads allowed)
__device__ __forceinline__ u32 lfind_ro(volatile lds_u32* par, u32 x) {
    u32 p;
    while ((p = par[x]) != x) x = p;
    return x;
}

__device__ __forceinline__ void lunion(u32* par_, u32 a, u32 b) {
    lds_u32* par = as_lds(par_);
    volatile lds_u32* vp = par;
    bool done;
    do {
        a = lfind(vp, a);
        b = lfind(vp, b);
        if (a < b) {
            u32 old = __hip_atomic_fetch_min(&par[b], a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            done = (old == b);
            b = old;
        } else if (b < a) {
            u32 old = __hip_atomic_fetch_min(&par[a], b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            done = (old == a);
            a = old;
        } else {
            done = true;
        }
    } while (!done);
}

// ---- global union-find over nodes, agent-coherent accesses ----
__device__ __forceinline__ u32 gload(u32* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void gstore(u32* p, u32 v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

__device__ __forceinline__ u32 gfind(u32* P, u32 x) {
    while (true) {
        u32 p = gload(P + x);
        if (p == x) return x;
        u32 gp = gload(P + p);
        if (gp == p) return p;
        gstore(P + x, gp);        // path halving: only ever points x at an ancestor
        x = gp;
    }
}

// Link the root with the larger key under the root with the smaller key.  Keys are
// unique per root, so the final root of a set is its minimum-key node.
__device__ __forceinline__ void gunion(u32* P, const u64* K, u32 a, u32 b) {
    while (true) {
        a = gfind(P, a);
        b = gfind(P, b);
        if (a == b) return;
        if (K[a] < K[b]) { u32 t = a; a = b; b = t; }
        u32 old = atomicCAS(P + a, a, b);
        if (old == a) return;
    }
}

// grid-stride loop for 1-D element kernels (grids are capped: a launch may not exceed 2^32 threads)
#define CC_FOR(i, n) \
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (int64_t)(n); i += (int64_t)gridDim.x * blockDim.x)

// the roots of a and b, both walks advancing together (their loads in flight at once; path
// halving as gfind)
__device__ __forceinline__ void gfind2(u32* P, u32& a, u32& b) {
    while (true) {
        const u32 pa = gload(P + a), pb = gload(P + b);
        const bool da = pa == a, db = pb == b;
        if (da && db) return;
        const u32 ga = da ? a : gload(P + pa), gb = db ? b : gload(P + pb);
        if (!da) {
            if (ga != pa) gstore(P + a, ga);
            a = ga;
        }
        if (!db) {
            if (gb != pb) gstore(P + b, gb);
            b = gb;
        }
    }
}

// gunion for two nodes whose roots were just found (usually still roots: one round of loads)
__device__ __forceinline__ void gunion_roots(u32* P, const u64* K, u32 a, u32 b) {
    while (true) {
        gfind2(P, a, b);
        if (a == b) return;
        const u64 ka = K[a], kb = K[b];
        if (ka < kb) { const u32 t = a; a = b; b = t; }
        if (atomicCAS(P + a, a, b) == a) return;
    }
}

// ---- wave-level scan and reductions by DPP (row shifts / row broadcasts of the VALU operand):
// no LDS round trip per step, where a shuffle (ds_bpermute) costs an LDS instruction and its
// latency at each of the six steps.  All 64 lanes must be active.
// dpp<CTRL, ROW, BANK>(old, x): x of the lane CTRL names; `old` where that lane is outside the
// row or the lane is masked off by the row / bank masks.
template <int CTRL, int ROW = 0xf, int BANK = 0xf>
__device__ __forceinline__ u32 dpp(u32 old, u32 x) {
    return (u32)__builtin_amdgcn_update_dpp((int)old, (int)x, CTRL, ROW, BANK, false);
}
constexpr int DPP_SHR1 = 0x111, DPP_SHR2 = 0x112, DPP_SHR3 = 0x113, DPP_SHR4 = 0x114, DPP_SHR8 = 0x118,
              DPP_BCAST15 = 0x142, DPP_BCAST31 = 0x143;

// sum of x over lanes 0..lane
__device__ __forceinline__ u32 wave_incl_sum(u32 x) {
    u32 y = x + dpp<DPP_SHR1>(0u, x);
    y += dpp<DPP_SHR2>(0u, x);
    y += dpp<DPP_SHR3>(0u, x);                 // lane: x over its 4-lane window of the row
    y += dpp<DPP_SHR4, 0xf, 0xe>(0u, y);       // lanes 4..15 of each row: 8-lane windows
    y += dpp<DPP_SHR8, 0xf, 0xc>(0u, y);       // lanes 8..15: the row's prefix
    y += dpp<DPP_BCAST15, 0xa>(0u, y);         // rows 1, 3: + the previous row's total
    y += dpp<DPP_BCAST31, 0xc>(0u, y);         // rows 2, 3: + the total of rows 0, 1
    return y;
}
// min (MAX = false) / max of x over the wave, in lane 63 (other lanes: partial results)
template <bool MAX>
__device__ __forceinline__ u32 wave_minmax_last(u32 x) {
    constexpr u32 id = MAX ? 0u : ~0u;
    auto op = [](u32 a, u32 b) { return MAX ? (a > b ? a : b) : (a < b ? a : b); };
    x = op(x, dpp<DPP_SHR1>(id, x));
    x = op(x, dpp<DPP_SHR2>(id, x));
    x = op(x, dpp<DPP_SHR4>(id, x));
    x = op(x, dpp<DPP_SHR8>(id, x));            // lane 15 of each row: the row's
    x = op(x, dpp<DPP_BCAST15, 0xa>(id, x));
    x = op(x, dpp<DPP_BCAST31, 0xc>(id, x));
    return x;
}
__device__ __forceinline__ u32 wave_min(u32 x) { return (u32)__builtin_amdgcn_readlane((int)wave_minmax_last<false>(x), 63); }
__device__ __forceinline__ u32 wave_max(u32 x) { return (u32)__builtin_amdgcn_readlane((int)wave_minmax_last<true>(x), 63); }

// ---- block-wide exclusive scan (NTHREADS threads) ----
__device__ __forceinline__ u32 block_excl_scan(u32 v, u32* scratch, u32* total) {
    const int tid = cc_tid(), lane = tid & 63, wave = tid >> 6;
    const u32 x = wave_incl_sum(v);
    if (lane == 63) scratch[wave] = x;
    __syncthreads();
    u32 base = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NTHREADS / 64; ++w) {
        u32 s = scratch[w];
        if (w < wave) base += s;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return base + x - v;
}

}  // namespace cc
