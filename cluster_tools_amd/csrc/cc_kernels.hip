// cc_kernels.hip -- gfx950 kernels of the thresholded connected-components path.
//
// Pipeline (one launch each; DESIGN.md §3 has the roofline per kernel):
//   k_block_stats   per-block min / max / NaN of the f32 input            (volume_utils.py:98-105)
//   k_block_params  per-block foreground interval in float order          (block_components.py:161-173)
//   k_pass1         threshold+mask -> bit rows -> tile CCL in LDS -> nodes, face planes
//   k_stitch<0>     26-connected unions across tile seams inside a block   (= block-local components)
//   k_collect_roots block-local roots -> (block, first voxel) sort keys
//   [radix sort]    -> skimage's raster first-occurrence numbering per block (block_components.py:179)
//   k_segments / k_values / [scan] / k_assign_rid   merge_offsets.py:104-120 on the device
//   k_stitch<1>     6-connected unions across block faces                 (block_faces.py:87-137,
//                                                                          merge_assignments.py:105-130)
//   k_lut           the 'assignments' LUT (min-id representative)
//   k_finalize      final label per node
//   k_pass2         bit rows -> tile CCL recomputed in LDS -> uint64 labels (write.py:185-202)
#include "cc_common.hpp"
#include "cc_rows.hpp"

namespace cc {

// ------------------------------------------------------------------------------------------
// direction tables for the 13 lex-negative cube neighbours (dz, dy, dx)
// cube mask bit index = lz*4 + ly*2 + lx
// ------------------------------------------------------------------------------------------
__host__ __device__ constexpr u32 sel_bits(int sz, int sy, int sx) {
    // s: 0 -> local 0 only, 1 -> local 1 only, 2 -> both
    u32 m = 0;
    for (int lz = 0; lz < 2; ++lz)
        for (int ly = 0; ly < 2; ++ly)
            for (int lx = 0; lx < 2; ++lx)
                if ((sz == 2 || sz == lz) && (sy == 2 || sy == ly) && (sx == 2 || sx == lx))
                    m |= 1u << (lz * 4 + ly * 2 + lx);
    return m;
}
__host__ __device__ constexpr int self_sel(int d) { return d < 0 ? 0 : d > 0 ? 1 : 2; }
__host__ __device__ constexpr int nbr_sel(int d) { return d < 0 ? 1 : d > 0 ? 0 : 2; }
// 4-bit face selection (layout p*2 + q)
__host__ __device__ constexpr u32 fsel(int sp, int sq) {
    u32 m = 0;
    for (int p = 0; p < 2; ++p)
        for (int q = 0; q < 2; ++q)
            if ((sp == 2 || sp == p) && (sq == 2 || sq == q)) m |= 1u << (p * 2 + q);
    return m;
}

#define CC_DIRS(X)                                                                            \
    X(-1, -1, -1) X(-1, -1, 0) X(-1, -1, 1) X(-1, 0, -1) X(-1, 0, 0) X(-1, 0, 1) X(-1, 1, -1) \
    X(-1, 1, 0) X(-1, 1, 1) X(0, -1, -1) X(0, -1, 0) X(0, -1, 1) X(0, 0, -1)
// the same without (0, 0, -1), which the x-runs cover
#define CC_DIRS12(X)                                                                          \
    X(-1, -1, -1) X(-1, -1, 0) X(-1, -1, 1) X(-1, 0, -1) X(-1, 0, 0) X(-1, 0, 1) X(-1, 1, -1) \
    X(-1, 1, 0) X(-1, 1, 1) X(0, -1, -1) X(0, -1, 0) X(0, -1, 1)

// ------------------------------------------------------------------------------------------
// Tile CCL in LDS.
//
// Bit rows use the SPLIT representation: one 64-bit word per voxel row (z, y) of the tile, low
// half = the even voxels (bit cx <-> x = 2 cx), high half = the odd voxels (bit cx <-> x = 2cx+1),
// so every cube-level mask is a 32-bit word with bit cx <-> cube cx (load_rows loads lane = x
// and splits each row once, split_row).
//
// A cube row (fixed cz, cy) holds 32 cubes of 2x2x2 voxels; all foreground voxels of a cube are
// mutually 26-adjacent.  Consecutive cubes are 26-linked along x iff the left one has a voxel at
// local x = 1 and the right one at local x = 0: E = H & (L >> 1) with L / H the OR of the row's
// even / odd halves.  Maximal x-linked sequences ("runs", up to 32 per cube row) are the
// union-find nodes, numbered in cube order (run id = first run id of the row + rank of its start
// among the row's run starts), so the root of a component -- its smallest run id -- is its first
// run in cube order (deterministic).  For each of the 12 other lex-negative cube directions the
// cube pairs are a 32-bit mask per pair of cube rows; a pair implied by the runs and the pair one
// cube to the left is dropped, only the rest reach the LDS union-find.
//
// After tile_ccl: par[run] = root | k << 16 for every run, k in [0, R) the component's compact
// index (roots in cube order).
// ------------------------------------------------------------------------------------------
// redo flags of the one-read-back schedule (scalars[3] of a run; bits of a shard's seam-pair
// header): the launch sequence enqueued without read-backs was not valid for this input, and the
// run is redone by the host-synchronised schedule (results never depend on which one ran)
constexpr u64 RF_BIG = 1;       // some block needs the global-memory stitch fallback
constexpr u64 RF_ROOTS = 2;     // more block-local roots than the root arrays hold
constexpr u64 RF_CUBES = 4;     // the slab's ids do not fit the 28-bit cube form of its top plane
constexpr u64 RF_PAIRS = 8;     // more seam pairs than the pair buffer holds
constexpr u64 RF_IOVF = 16;     // some tile's block-face pair list overflowed (the global-memory
                                // inter stitch, k_stitch<true>, runs in the synchronised schedule)

// the run's device scalars: [0] sum of block values, [1] components owned, [2] block-local roots,
// [3] redo flags, [5] seam pairs appended
constexpr int SCALARS = 8;
constexpr int64_t SEAM_SET = 1 << 16;   // slots of the seam pair hash set (k_seam_pairs, k_seam_cube_pairs)

constexpr int NCROW = CZ * CY;          // cube rows per tile
constexpr int NRUN = NCROW * CX;        // a run per occupied cube at most (adjacent cubes need not link)
static_assert(NTHREADS == 4 * NCROW, "tile_ccl maps one thread to each quarter cube row");

__device__ __forceinline__ u32 lo32(u64 w) { return (u32)w; }
__device__ __forceinline__ u32 hi32(u64 w) { return (u32)(w >> 32); }
// mask of bits 0..b (b in [0, 31])
__device__ __forceinline__ u32 mask_le(int b) { return (u32)((2ull << b) - 1); }

// OR of the voxel rows of a cube row whose (lz, ly) match selections (sz, sy); a[lz*2+ly]
__device__ __forceinline__ u64 pick_rows(const u64 a[4], int sz, int sy) {
    u64 u = 0;
    if (sz != 1 && sy != 1) u |= a[0];
    if (sz != 1 && sy != 0) u |= a[1];
    if (sz != 0 && sy != 1) u |= a[2];
    if (sz != 0 && sy != 0) u |= a[3];
    return u;
}

struct TileCCL {
    u32 B[NCROW];          // run starts of each cube row (bit cx)
    u32 E[NCROW];          // x-links: bit cx iff cube cx is 26-linked to cube cx + 1
    u32 roff[NCROW];       // run id of each cube row's first run
    u32 scratch[8];
    u32 par[NRUN];         // union-find over run ids, then root | k << 16
};

__device__ __forceinline__ void load_row4(const u64* rows, int row, u64 a[4]) {
    const int cz = row / CY, cy = row % CY;
#pragma unroll
    for (int j = 0; j < 4; ++j) a[j] = rows[(2 * cz + (j >> 1)) * TY + 2 * cy + (j & 1)];
}

// run id of occupied cube cx of cube row `row`
__device__ __forceinline__ u32 run_of(const TileCCL& T, int row, int cx) {
    return T.roff[row] + (u32)__popc(T.B[row] & mask_le(cx)) - 1;
}
// run id of the run starting at cube cx0 (a set bit of B)
__device__ __forceinline__ u32 run_at(const TileCCL& T, int row, int cx0) {
    return T.roff[row] + (u32)__popc(T.B[row] & ((1u << cx0) - 1));
}

// Thread (row = tid / 4, q = tid % 4) owns the run starts in cubes [8q, 8q + 8) of cube row `row`,
// so the per-run phases keep all 8 waves busy; tid order is run-id order.
#ifndef CC_CCL_LIST
#define CC_CCL_LIST 1
#endif
// list (nullable, LDS, capacity NRUN): phase 2 first lists its union pairs, then every thread takes
// an equal share of the list (each thread's own contacts vary from none to dozens: processed in
// place they leave most lanes idle and the barrier waiting for the busiest row)
// firstv (nullable, LDS, may alias list): firstv[k] = the first voxel (tile raster index) of
// component k, computed in phase 5 from each run's first voxel (pass 1's keys).
template <int STOP = 0>   // ablation harness only: return after phase STOP (1..3; 4: pair list only)
__device__ __forceinline__ u32 tile_ccl(const u64* rows, TileCCL& T, u32* list = nullptr, u32* firstv = nullptr) {
    const int tid = cc_tid();
    const int qrow = tid >> 2, q = tid & 3;
    u32* par = T.par;
    // 1. runs per cube row, run ids (scan of the run counts), every run its own parent
    u32 Bq;
    {
        u64 a[4];
        load_row4(rows, qrow, a);
        const u32 L = lo32(a[0] | a[1] | a[2] | a[3]), H = hi32(a[0] | a[1] | a[2] | a[3]);
        const u32 E = H & (L >> 1);
        const u32 B = (L | H) & ~(E << 1);
        u32 nrun = 0;
        const u32 off = block_excl_scan(q == 0 ? (u32)__popc(B) : 0u, T.scratch, &nrun);
        if (q == 0) { T.B[qrow] = B; T.E[qrow] = E; T.roff[qrow] = off; }
        for (u32 i = tid; i < nrun; i += NTHREADS) par[i] = i;
        Bq = B & (0xFFu << (8 * q));
    }
    __syncthreads();
    if (STOP == 1) return 0;
    // 2. unions between runs of neighbouring cube rows: thread = (row, direction group)
    if (CC_CCL_LIST && list) {
        const int row = tid % NCROW, grp = tid / NCROW;          // grp is uniform per 2 waves
        const int cz = row / CY, cy = row % CY;
        const int dz = grp == 3 ? 0 : -1, dy = grp == 3 ? -1 : grp - 1;
        const int bz = cz + dz, by = cy + dy;
        const bool ok = bz >= 0 && by >= 0 && by < CY;
        const int rowb = ok ? bz * CY + by : row;
        u32 M[3] = {0u, 0u, 0u};
        u32 BA = 0, BB = 0, ra0 = 0, rb0 = 0, cnt = 0;
        if (ok) {
            u64 a[4], b[4];
            load_row4(rows, row, a);
            load_row4(rows, rowb, b);
            const int szs = dz < 0 ? 0 : 2, szn = dz < 0 ? 1 : 2;
            const int sys = dy < 0 ? 0 : dy > 0 ? 1 : 2, syn = dy < 0 ? 1 : dy > 0 ? 0 : 2;
            const u64 ua = pick_rows(a, szs, sys), ub = pick_rows(b, szn, syn);
            const u32 ua0 = lo32(ua), ua1 = hi32(ua), ub0 = lo32(ub), ub1 = hi32(ub);
            const u32 Ea = T.E[row], Eb = T.E[rowb];
            BA = T.B[row]; BB = T.B[rowb]; ra0 = T.roff[row]; rb0 = T.roff[rowb];
            const u32 C0 = (ua0 | ua1) & (ub0 | ub1);
#pragma unroll
            for (int dx = -1; dx <= 1; ++dx) {
                const u32 C = dx < 0 ? ua0 & (ub1 << 1) : dx > 0 ? ua1 & (ub0 >> 1) : C0;
                const u32 ebs = dx < 0 ? Eb << 2 : dx > 0 ? Eb : Eb << 1;
                u32 red = (C << 1) & (Ea << 1) & ebs;
                if (dx > 0) red |= ((C0 >> 1) & Ea) | (C0 & Eb);
                if (dx < 0) red |= ((C0 & Ea) << 1) | (C0 & (Eb << 1));
                M[dx + 1] = C & ~red;
                cnt += (u32)__popc(M[dx + 1]);
            }
        }
        u32 total = 0;
        u32 pos = block_excl_scan(cnt, T.scratch, &total);
#pragma unroll
        for (int d = 0; d < 3; ++d)
            for (u32 m = M[d]; m; m &= m - 1) {
                const int cx = __builtin_ctz(m);
                const u32 ra = ra0 + (u32)__popc(BA & mask_le(cx)) - 1;
                const u32 rb = rb0 + (u32)__popc(BB & mask_le(cx + d - 1)) - 1;
                if (pos < (u32)NRUN) list[pos] = ra | (rb << 16);
                else lunion(par, ra, rb);                    // list full: in place
                ++pos;
            }
        __syncthreads();
        if (STOP == 4) return 0;       // ablation: the pair list without the unions
        const u32 nl = total < (u32)NRUN ? total : (u32)NRUN;
        for (u32 i = tid; i < nl; i += NTHREADS) {
            const u32 e = list[i];
            lunion(par, e & 0xFFFFu, e >> 16);
        }
    } else
    for (int w = tid; w < NCROW * 4; w += NTHREADS) {
        const int row = w % NCROW, grp = w / NCROW;          // grp is uniform per 2 waves
        const int cz = row / CY, cy = row % CY;
        const int dz = grp == 3 ? 0 : -1, dy = grp == 3 ? -1 : grp - 1;
        const int bz = cz + dz, by = cy + dy;
        if (bz < 0 || by < 0 || by >= CY) continue;
        const int rowb = bz * CY + by;
        u64 a[4], b[4];
        load_row4(rows, row, a);
        load_row4(rows, rowb, b);
        const int szs = dz < 0 ? 0 : 2, szn = dz < 0 ? 1 : 2;
        const int sys = dy < 0 ? 0 : dy > 0 ? 1 : 2, syn = dy < 0 ? 1 : dy > 0 ? 0 : 2;
        const u64 ua = pick_rows(a, szs, sys), ub = pick_rows(b, szn, syn);
        const u32 ua0 = lo32(ua), ua1 = hi32(ua), ub0 = lo32(ub), ub1 = hi32(ub);
        const u32 Ea = T.E[row], Eb = T.E[rowb];                  // bit cx: cube cx linked to cx + 1
        const u32 BA = T.B[row], BB = T.B[rowb], ra0 = T.roff[row], rb0 = T.roff[rowb];
        const u32 C0 = (ua0 | ua1) & (ub0 | ub1);                 // contacts (cx, cx)
#pragma unroll
        for (int dx = -1; dx <= 1; ++dx) {
            // own cube cx with neighbour cube cx + dx: own voxels facing -dx, neighbour voxels facing dx
            const u32 C = dx < 0 ? ua0 & (ub1 << 1) : dx > 0 ? ua1 & (ub0 >> 1) : C0;
            // implied unions: the same contact one cube to the left with both pairs of cubes linked,
            // and (dx != 0) a (cx, cx) contact next to it with the cubes in between linked
            const u32 ebs = dx < 0 ? Eb << 2 : dx > 0 ? Eb : Eb << 1;
            u32 red = (C << 1) & (Ea << 1) & ebs;
            if (dx > 0) red |= ((C0 >> 1) & Ea) | (C0 & Eb);
            if (dx < 0) red |= ((C0 & Ea) << 1) | (C0 & (Eb << 1));
            for (u32 m = C & ~red; m; m &= m - 1) {
                const int cx = __builtin_ctz(m);
                const u32 ra = ra0 + (u32)__popc(BA & mask_le(cx)) - 1;
                const u32 rb = rb0 + (u32)__popc(BB & mask_le(cx + dx)) - 1;
                lunion(par, ra, rb);
            }
        }
    }
    __syncthreads();
    if (STOP == 2) return 0;
    // 3. compress; count the roots of each quarter row.  The finds here must not compress
    // paths: a compressing find of another thread could store an intermediate ancestor into
    // par[r] after r's owner stored the root, and phase 5 would then read that ancestor's entry
    // (mid-update) as the root's -- a run silently landing in another component of the tile.
    // Without it every store to par[r] is the root itself, by r's owner only.
    const u32 r0 = T.roff[qrow];
    const u32 Brow = T.B[qrow];
    u32 n = 0;
    for (u32 m = Bq; m; m &= m - 1) {
        const u32 r = r0 + (u32)__popc(Brow & ((1u << __builtin_ctz(m)) - 1));
        const u32 root = lfind_ro(as_lds(par), r);
        par[r] = root;
        n += (root == r);
    }
    __syncthreads();
    if (STOP == 3) return 0;
    // 4. compact index k of every root, in run-id order; a root also records its cube layer cz in
    // bits 12-14 (run ids < 4096): the component's first voxel lies in that layer (the root is
    // its first run in cube order, so no run of it has a smaller cz), so phase 5 only offers
    // first voxels from runs of that layer
    static_assert(NRUN <= (1 << 12) && CZ <= 8, "root | cz << 12 | k << 16");
    u32 total = 0;
    {
        const u32 base = block_excl_scan(n, T.scratch, &total);
        u32 k = base;
        const u32 czb = (u32)(qrow / CY) << 12;
        for (u32 m = Bq; m; m &= m - 1) {
            const u32 r = r0 + (u32)__popc(Brow & ((1u << __builtin_ctz(m)) - 1));
            if (par[r] == r) par[r] = r | czb | (k++ << 16);
        }
        if (firstv)
            for (u32 i = tid; i < total; i += NTHREADS) firstv[i] = NONE;
    }
    __syncthreads();
    // 5. every run carries its component's k (and, for pass 1, offers its first voxel in raster
    // order -- the first sub-row (lz, ly) with a voxel in the run's cubes, then its smallest x)
    u64 a[4];
    u32 E = 0;
    if (firstv) {
        load_row4(rows, qrow, a);
        E = T.E[qrow];
    }
    const int cz = qrow / CY, cy = qrow % CY;
    for (u32 m = Bq; m; m &= m - 1) {
        const int c0 = __builtin_ctz(m);
        const u32 r = r0 + (u32)__popc(Brow & ((1u << c0) - 1));
        const u32 root = par[r] & 0xFFFu;
        const u32 pr = par[root];
        const u32 pk = pr & 0xFFFF0000u;
        if (root != r) par[r] = root | pk;
        if (firstv && ((pr >> 12) & 7u) == (u32)cz) {
            const int c1 = c0 + __builtin_ctz(~(E >> c0));                    // end cube
            const u32 M = mask_le(c1) & ~((1u << c0) - 1);
            u32 idx = NONE;
#pragma unroll
            for (int j = 3; j >= 0; --j) {
                const u32 ev = lo32(a[j]) & M, od = hi32(a[j]) & M;
                if (ev | od) {
                    const int xe = ev ? 2 * __builtin_ctz(ev) : TX, xo = od ? 2 * __builtin_ctz(od) + 1 : TX;
                    idx = (u32)(((2 * cz + (j >> 1)) * TY + 2 * cy + (j & 1)) * TX + (xe < xo ? xe : xo));
                }
            }
            atomicMin(&firstv[pk >> 16], idx);
        }
    }
    __syncthreads();
    return total;
}

// component index k of an occupied cube
__device__ __forceinline__ u32 cube_k(const TileCCL& T, int row, int cx) { return T.par[run_of(T, row, cx)] >> 16; }
__device__ __forceinline__ u32 cube_k(const TileCCL& T, int c) { return cube_k(T, c / CX, c % CX); }

// ------------------------------------------------------------------------------------------
// k_block_stats: per-block ordered min / max and NaN flag (for_tile_rows / stats_tile: cc_rows.hpp)
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(NTHREADS) void k_block_stats(Geom g, const float* __restrict__ in,
                                                          u32* smin, u32* smax, u32* sflag) {
    __shared__ u32 red[3][NTHREADS / 64];
    stats_tile(g, tile_info(g, blockIdx.x), in, smin, smax, sflag, red);
}

// ------------------------------------------------------------------------------------------
// k_block_params: exact foreground interval per block.  f(x) = fl32(fl32(x - mn) / m) is
// monotone non-decreasing in x for finite blocks, so {x : f(x) OP thr} is an interval in float
// order; it is found by binary search with the reference's own arithmetic.  Blocks with +-inf
// fall back to the exact per-voxel expression; blocks with NaN have no foreground.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float norm_at(u32 o, float mn, float m) {
    float y = __uint_as_float(ord2f(o)) - mn;
    if (m > 0.0f) y = y / m;
    return y;
}

__device__ BlockParam block_param(u32 vmin, u32 vmax, u32 vflag, float thr, int mode) {
    BlockParam p;
    p.kind = BP_EMPTY; p.lo = 1; p.hi = 0; p.pad = 0;
    const u32 omn = vmin, omx = vmax;
    const float mn = __uint_as_float(ord2f(omn)), mx = __uint_as_float(ord2f(omx));
    p.mn = mn;
    p.m = 0.0f;
    if (vflag & 1u) return p;                                  // NaN anywhere: numpy min is NaN
    if (isinf(mn) || isinf(mx)) {
        p.kind = BP_EXACT;
        p.m = isinf(mn) ? __uint_as_float(0x7FC00000u) : mx - mn;
        return p;
    }
    const float m = mx - mn;
    p.m = m;
    if (mode == MODE_GREATER) {
        if (norm_at(omx, mn, m) > thr) {
            u32 L = omn, H = omx;
            while (L < H) { u32 M = L + (H - L) / 2; if (norm_at(M, mn, m) > thr) H = M; else L = M + 1; }
            p.kind = BP_INTERVAL; p.lo = L; p.hi = omx;
        }
    } else if (mode == MODE_LESS) {
        if (norm_at(omn, mn, m) < thr) {
            u32 L = omn, H = omx;
            while (L < H) { u32 M = L + (H - L + 1) / 2; if (norm_at(M, mn, m) < thr) L = M; else H = M - 1; }
            p.kind = BP_INTERVAL; p.lo = omn; p.hi = L;
        }
    } else {
        if (norm_at(omx, mn, m) >= thr && norm_at(omn, mn, m) <= thr) {
            u32 L = omn, H = omx;
            while (L < H) { u32 M = L + (H - L) / 2; if (norm_at(M, mn, m) >= thr) H = M; else L = M + 1; }
            const u32 a = L;
            L = omn; H = omx;
            while (L < H) { u32 M = L + (H - L + 1) / 2; if (norm_at(M, mn, m) <= thr) L = M; else H = M - 1; }
            const u32 bb = L;
            if (a <= bb) { p.kind = BP_INTERVAL; p.lo = a; p.hi = bb; }
        }
    }
    return p;
}


__global__ void k_block_params(int64_t nb, const u32* smin, const u32* smax, const u32* sflag,
                               float thr, int mode, BlockParam* bp) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b < nb) bp[b] = block_param(smin[b], smax[b], sflag[b], thr, mode);
}

// ------------------------------------------------------------------------------------------
// shared: load the tile's foreground bit rows (threshold + mask) into LDS
// ------------------------------------------------------------------------------------------
// Bit rows of the tile into LDS: the wave's 64 row masks are collected one per lane
// (writelane) and stored with one 8-B LDS write per lane.  Rows outside the tile stay 0.
// The v_writelane asm relies on wave-uniform control flow here (the wave index and the tile are
// SGPR values); under a branch the compiler treats as divergent it produced wrong rows (k_seams).
// lane j of (lo, hi) := the SGPR pair (blo, bhi).  The s_nop: the ballot feeding blo is often
// the VALU instruction right before, and v_writelane reading an SGPR a VALU has just written
// took the stale value (lanes 0-31 of rows lost in k_spec); inline asm is opaque to the
// compiler's hazard recognizer, so the wait states are spelled out.  j must be a constant.
#define CC_WRITELANE2(lo, hi, blo, bhi, j)                                                        \
    asm("s_nop 3\n\tv_writelane_b32 %0, %2, %4\n\tv_writelane_b32 %1, %3, %4"                      \
        : "+v"(lo), "+v"(hi)                                                                      \
        : "s"(blo), "s"(bhi), "i"(j))

// natural bit row (bit x <-> voxel x) -> split row (even voxels low, odd voxels high): the
// inverse perfect shuffle, once per row after the (coalesced, lane = x) loads
__device__ __forceinline__ u64 split_row(u64 x) {
    u64 t;
    t = (x ^ (x >> 1)) & 0x2222222222222222ull;  x ^= t ^ (t << 1);
    t = (x ^ (x >> 2)) & 0x0C0C0C0C0C0C0C0Cull;  x ^= t ^ (t << 2);
    t = (x ^ (x >> 4)) & 0x00F000F000F000F0ull;  x ^= t ^ (t << 4);
    t = (x ^ (x >> 8)) & 0x0000FF000000FF00ull;  x ^= t ^ (t << 8);
    t = (x ^ (x >> 16)) & 0x00000000FFFF0000ull; x ^= t ^ (t << 16);
    return x;
}

template <bool HAS_MASK>
__device__ __forceinline__ void load_rows(const Geom& g, const TileInfo& ti, const float* __restrict__ in,
                                          const u8* __restrict__ mask, const BlockParam& p, float thr,
                                          int mode, u64* rows) {
    const int lane = cc_tid() & 63, wave = wave_id();
    const u64 lanes = ti.lx >= 64 ? ~0ull : ((1ull << ti.lx) - 1);
    u32 mlo = 0, mhi = 0;                   // lane j: row mask of slot j
    auto put = [&](int j, u64 bal) {
        bal &= lanes;
        const u32 blo = (u32)bal, bhi = (u32)(bal >> 32);
        CC_WRITELANE2(mlo, mhi, blo, bhi, j);
    };
    if (p.kind == BP_INTERVAL) {
        // lo <= ord(x) <= hi as two float compares: the interval never splits -0 from +0 (the
        // predicate is the same for both) and interval blocks hold no NaN
        const float flo = __uint_as_float(ord2f(p.lo)), fhi = __uint_as_float(ord2f(p.hi));
        for_tile_rows<HAS_MASK>(g, ti, in, mask, [&](int j, float x, u32 mk) {
            u64 bal = __ballot(x >= flo) & __ballot(x <= fhi);
            if (HAS_MASK) bal &= __ballot(mk != 0);
            put(j, bal);
        });
    } else if (p.kind == BP_EXACT) {
        for_tile_rows<HAS_MASK>(g, ti, in, mask, [&](int j, float x, u32 mk) {
            bool fg = exact_pred(x, p.mn, p.m, thr, mode);
            if (HAS_MASK) fg = fg && mk != 0;
            put(j, __ballot(fg));
        });
    }
    const int r = slot_row(lane, wave);
    if (r / TY < ti.lz && r % TY < ti.ly) rows[r] = split_row(((u64)mhi << 32) | mlo);
}

// bit i of x (i < 16) -> bit 2i
__device__ __forceinline__ u32 spread2(u32 x) {
    x &= 0xFFFFu;
    x = (x | (x << 8)) & 0x00FF00FFu;
    x = (x | (x << 4)) & 0x0F0F0F0Fu;
    x = (x | (x << 2)) & 0x33333333u;
    x = (x | (x << 1)) & 0x55555555u;
    return x;
}

// voxel x of a split bit row
__device__ __forceinline__ u32 vbit(u64 w, int x) { return (u32)(w >> ((x & 1) * 32 + (x >> 1))) & 1u; }
// the two voxels (2cx, 2cx + 1) of cube column cx of a split row, as bits 0 / 1
__device__ __forceinline__ u32 vpair(u64 w, int cx) { return ((u32)(w >> cx) & 1u) | (((u32)(w >> (32 + cx)) & 1u) << 1); }


// Face entries 2w and 2w + 1 (one 32-bit word of the face planes): two neighbouring cubes of one
// face, so their voxel rows and cube rows are read once.  Rows and bits outside the tile are 0,
// so no extent test is needed (an entry without face voxels is 0).
__device__ __forceinline__ u32 face_k(const TileCCL& T, int row, int cx) {
    return T.par[T.roff[row] + (u32)__popc(T.B[row] & mask_le(cx)) - 1] >> 16;
}
__device__ __forceinline__ u32 face_word(int w, const u64* rows, const TileCCL& T, const TileInfo& ti) {
    const int i = 2 * w;
    u32 b0, b1;
    int row0, row1, c0, c1;
    if (i < F_YLO) {                       // z faces: (cy, cx), (cy, cx + 1); bits (y-local)*2 + (x-local)
        const bool hi = i >= F_ZHI;
        const int e = hi ? i - F_ZHI : i;
        const int cy = e / CX, cx = e % CX;
        const int z = hi ? ti.lz - 1 : 0;
        const u64 r0 = rows[z * TY + 2 * cy], r1 = rows[z * TY + 2 * cy + 1];
        b0 = vpair(r0, cx) | (vpair(r1, cx) << 2);
        b1 = vpair(r0, cx + 1) | (vpair(r1, cx + 1) << 2);
        row0 = row1 = (z >> 1) * CY + cy;
        c0 = cx; c1 = cx + 1;
    } else if (i < F_XLO) {                // y faces: (cz, cx), (cz, cx + 1); bits (z-local)*2 + (x-local)
        const bool hi = i >= F_YHI;
        const int e = hi ? i - F_YHI : i - F_YLO;
        const int cz = e / CX, cx = e % CX;
        const int y = hi ? ti.ly - 1 : 0;
        const u64 r0 = rows[(2 * cz) * TY + y], r1 = rows[(2 * cz + 1) * TY + y];
        b0 = vpair(r0, cx) | (vpair(r1, cx) << 2);
        b1 = vpair(r0, cx + 1) | (vpair(r1, cx + 1) << 2);
        row0 = row1 = cz * CY + (y >> 1);
        c0 = cx; c1 = cx + 1;
    } else {                               // x faces: (cz, cy), (cz, cy + 1); bits (z-local)*2 + (y-local)
        const bool hi = i >= F_XHI;
        const int e = hi ? i - F_XHI : i - F_XLO;
        const int cz = e / CY, cy = e % CY;
        const int x = hi ? ti.lx - 1 : 0;
        const u64* r = rows + (2 * cz) * TY + 2 * cy;
        b0 = vbit(r[0], x) | (vbit(r[1], x) << 1) | (vbit(r[TY], x) << 2) | (vbit(r[TY + 1], x) << 3);
        b1 = vbit(r[2], x) | (vbit(r[3], x) << 1) | (vbit(r[TY + 2], x) << 2) | (vbit(r[TY + 3], x) << 3);
        row0 = cz * CY + cy;
        row1 = row0 + 1;
        c0 = c1 = x >> 1;
    }
    const u32 e0 = b0 ? face_k(T, row0, c0) | (b0 << FK_BITS) : 0u;
    const u32 e1 = b1 ? face_k(T, row1, c1) | (b1 << FK_BITS) : 0u;
    return e0 | (e1 << 16);
}

// ------------------------------------------------------------------------------------------
// k_pass1: bit rows, tile-local components, their first voxels, face planes
// ------------------------------------------------------------------------------------------
// LDS of one pass-1 tile
struct Pass1LDS {
    u64 rows[NROWS];
    TileCCL T;
    u32 key[NRUN];            // first voxel (tile raster index) of each component (<= one per run)
};

template <int ABL>
__device__ __forceinline__ void pass1_finish(const Geom& g, int64_t t, const TileInfo& ti, u64* BITS, face_t* FACES,
                                             u32* COUNT, u32* P, u64* KEY, Pass1LDS& L, bool write,
                                             u8* fchg = nullptr, int empty = -1);

// Pass 1 of tile t (block parameters p): bit rows -> BITS, tile CCL -> COUNT, nodes (P, KEY),
// face planes.  ABL (kernel ablation harness tools/ablate.hip only; 0 in the library): stop
// after phase ABL (1 bits, 2 CCL, 3 first voxels; 11..13 inside the CCL after its phase 1..3).
template <bool HAS_MASK, int ABL = 0>
__device__ __forceinline__ void pass1_tile(const Geom& g, int64_t t, const TileInfo& ti, const BlockParam& p,
                                           const float* __restrict__ in, const u8* __restrict__ mask, float thr,
                                           int mode, u64* BITS, face_t* FACES, u32* COUNT, u32* P, u64* KEY,
                                           Pass1LDS& L, bool write = true, u8* fchg = nullptr) {
    const int tid = cc_tid();
    for (int i = tid; i < NROWS; i += NTHREADS) L.rows[i] = 0;
    __syncthreads();
    if (p.kind != BP_EMPTY) load_rows<HAS_MASK>(g, ti, in, mask, p, thr, mode, L.rows);
    __syncthreads();
    pass1_finish<ABL>(g, t, ti, BITS, FACES, COUNT, P, KEY, L, write, fchg);
}

// pass 1's BITS / FACES stores, non-temporal (CC_SPEC_NT=0 for A/B: plain stores; C3 on a fast box
// k_spec 3.140-3.148 -> 3.113-3.122 ms, C4 unchanged: profiles/r05_ab_spec_nt.txt)
#ifndef CC_SPEC_NT
#define CC_SPEC_NT 1
#endif
template <class T>
__device__ __forceinline__ void spec_store(T* p, T v) {
    if (CC_SPEC_NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// Pass 1 after the bit rows are in L.rows (and a barrier): BITS, tile CCL, COUNT, nodes, faces.
// fchg (k_fix): fchg[t] = 1 when the new face planes differ from the ones in FACES (the seams
// that read them must be redone; unchanged faces leave every seam list as it was).
// empty: whether the tile has no foreground voxel, if the caller knows (k_spec reads it off its
// statistics barrier); -1: decided here (one more barrier)
template <int ABL>
__device__ __forceinline__ void pass1_finish(const Geom& g, int64_t t, const TileInfo& ti, u64* BITS, face_t* FACES,
                                             u32* COUNT, u32* P, u64* KEY, Pass1LDS& L, bool write, u8* fchg,
                                             int empty) {
    u64* rows = L.rows;
    TileCCL& T = L.T;
    u32* key = L.key;
    const int tid = cc_tid();
    // An empty tile (no foreground voxel: a masked-out or all-background region) stores no bit
    // rows -- k_pass2 writes its zeros without them -- and skips the tile CCL; its faces are
    // stored as zeros (their readers take them as they are).
    static_assert(NROWS == NTHREADS, "one bit row per thread");
    if (ABL == 0 && write && (empty >= 0 ? empty != 0 : !__syncthreads_or(rows[tid] != 0))) {
        if (tid == 0) COUNT[t] = 0;
        u32* FW = (u32*)(FACES + t * FACE_STRIDE);
        const bool two = NTHREADS + tid < FACE_STRIDE / 2;
        if (fchg) {
            const bool diff = FW[tid] != 0u || (two && FW[NTHREADS + tid] != 0u);
            if (__syncthreads_or(diff) && tid == 0) fchg[t] = 1;
        }
        FW[tid] = 0u;
        if (two) FW[NTHREADS + tid] = 0u;
        return;
    }
    // (ABL 20 / 21 / 22: the whole pass without the BITS / FACES / both stores -- the store-volume
    // ablation of tools/ablate.hip)
    if (write && ABL != 20 && ABL != 22)
        for (int i = tid; i < NROWS; i += NTHREADS) spec_store(BITS + t * NROWS + i, rows[i]);
    if (ABL == 1) return;
    if constexpr (ABL >= 10 && ABL < 20) { tile_ccl<ABL - 10>(rows, T, key, key); return; }
    const u32 R = tile_ccl(rows, T, key, key);      // key[k] = first voxel of component k
    if (ABL == 2) { if (tid == 0) COUNT[t] = R; return; }
    if (tid == 0 && write) COUNT[t] = R;
    if (ABL == 3 || !write) return;
    const u32 base = (u32)(t * g.cap);
    for (u32 k = tid; k < R; k += NTHREADS) {
        const u32 node = base + k;
        const u32 idx = key[k];
        const int lz = idx / (TY * TX), ly = (idx / TX) % TY, lx = idx % TX;
        P[node] = node;
        KEY[node] = ((u64)(g.zoff + ti.z0 + lz) * (u64)g.Y + (u64)(ti.y0 + ly)) * (u64)g.X + (u64)(ti.x0 + lx);
    }
    u32* FW = (u32*)(FACES + t * FACE_STRIDE);          // two 16-bit entries per store
    static_assert(F_YLO == 2 * NTHREADS && FACE_STRIDE / 2 <= 2 * NTHREADS, "face words: z faces, then y / x");
    const u32 w0 = face_word(tid, rows, T, ti);
    const bool two = NTHREADS + tid < FACE_STRIDE / 2;
    const u32 w1 = two ? face_word(NTHREADS + tid, rows, T, ti) : 0u;
    if (fchg) {
        const bool diff = FW[tid] != w0 || (two && FW[NTHREADS + tid] != w1);
        if (__syncthreads_or(diff) && tid == 0) fchg[t] = 1;
    }
    if (ABL == 21 || ABL == 22) {          // ablation: faces computed, not stored
        if (__syncthreads_or(w0 == 0x12345678u && w1 == 0x9ABCDEF0u) && tid == 0) COUNT[t] = R + 1;
        return;
    }
    spec_store(FW + tid, w0);
    if (two) spec_store(FW + NTHREADS + tid, w1);
}

// k_pass1: one workgroup per tile, block parameters precomputed (ablation harness; the library
// runs pass 1 inside k_spec / k_fix)
template <bool HAS_MASK, int ABL = 0>
__global__ __launch_bounds__(NTHREADS) void k_pass1(Geom g, const float* __restrict__ in,
                                                    const u8* __restrict__ mask, const BlockParam* bp,
                                                    float thr, int mode, u64* BITS, face_t* FACES,
                                                    u32* COUNT, u32* P, u64* KEY) {
    __shared__ Pass1LDS L;
    const int64_t t = blockIdx.x;
    const TileInfo ti = tile_info(g, t);
    pass1_tile<HAS_MASK, ABL>(g, t, ti, uniform_bp(bp[ti.block]), in, mask, thr, mode, BITS, FACES, COUNT, P, KEY, L);
}

// global tile id of local tile lt (z-major inside the block) of block b
__device__ __forceinline__ int64_t block_tile(const Geom& g, int64_t b, int lt) {
    const int bx = (int)(b % g.nb[2]), by = (int)((b / g.nb[2]) % g.nb[1]), bz = (int)(b / ((int64_t)g.nb[2] * g.nb[1]));
    const int nx = g.btn[2][bx], ny = g.btn[1][by];
    const int lx = lt % nx, ly = (lt / nx) % ny, lz = lt / (nx * ny);
    return ((int64_t)(g.bt0[0][bz] + lz) * g.nt[1] + (g.bt0[1][by] + ly)) * g.nt[2] + (g.bt0[2][bx] + lx);
}

// tile tables read after stores come back in VGPRs (vector loads); the values are
// workgroup-uniform, so move them to SGPRs
__device__ __forceinline__ TileInfo uniform_ti(TileInfo ti) {
    ti.iz = __builtin_amdgcn_readfirstlane(ti.iz); ti.iy = __builtin_amdgcn_readfirstlane(ti.iy);
    ti.ix = __builtin_amdgcn_readfirstlane(ti.ix); ti.z0 = __builtin_amdgcn_readfirstlane(ti.z0);
    ti.y0 = __builtin_amdgcn_readfirstlane(ti.y0); ti.x0 = __builtin_amdgcn_readfirstlane(ti.x0);
    ti.lz = __builtin_amdgcn_readfirstlane(ti.lz); ti.ly = __builtin_amdgcn_readfirstlane(ti.ly);
    ti.lx = __builtin_amdgcn_readfirstlane(ti.lx);
    const u64 b = (u64)ti.block;
    ti.block = (int64_t)(((u64)__builtin_amdgcn_readfirstlane((u32)(b >> 32)) << 32) | __builtin_amdgcn_readfirstlane((u32)b));
    return ti;
}

// ------------------------------------------------------------------------------------------
// Speculative front (the library's path): block statistics and pass 1 from ONE read of the input.
//
// The foreground of a block is an interval of the float order fixed by the block's min / max
// (k_block_params), which are only known once the whole block has been read.  k_sample guesses
// each block's interval from a sparse sample (1/512 of the block, k_sample + k_guess); k_spec then reads every tile
// once, accumulating the exact block statistics AND labelling the tile (pass 1) with the guessed
// interval [lg, hg], and records per tile the nearest values on both sides of each guessed bound:
//   TB = { max ord < lg, min ord >= lg, max ord <= hg, min ord > hg }  (masked-out voxels excluded).
// With the exact interval [lt, ht] (k_block_params) a tile's bits are the exact bits iff no voxel
// lies between lg and lt nor between hg and ht -- decided from TB alone (spec_valid).  k_verify
// k_verify lists the tiles that fail and k_fix relabels them from the input with the exact interval.
// A one-sided interval is kept open to the end of the order (widen): it then differs from the
// exact one only in its finite bound.  On quantized data the sampled extremes are usually the
// block's and the guess is exact; on continuous data it misses the exact bound by about the
// extremes' sampling error, and only tiles holding a voxel in between are relabelled (1 % of the
// C3 tiles with the dithered map).  Results never depend on the guess; only the k_fix work does.
// ------------------------------------------------------------------------------------------
// one voxel row per 4 planes x 16 rows of a block (1/64 of it: on continuous data the guessed
// bounds miss the exact ones by about the extremes' sampling error, so a denser sample leaves
// fewer tiles with a voxel in between; 1/512 left 8 % of the C3 tiles to k_fix)
constexpr int SAMPLE_DZ = 4, SAMPLE_DY = 16;

__device__ __forceinline__ void block_extent(const Geom& g, int64_t b, int e0[3], int el[3]) {
    const int bi[3] = {(int)(b / ((int64_t)g.nb[2] * g.nb[1])), (int)((b / g.nb[2]) % g.nb[1]), (int)(b % g.nb[2])};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const int t0 = g.bt0[a][bi[a]], t1 = t0 + g.btn[a][bi[a]] - 1;
        e0[a] = g.tstart[a][t0];
        el[a] = g.tstart[a][t1] + g.tlen[a][t1] - e0[a];
    }
}

__device__ __forceinline__ BlockParam widen(BlockParam p, int mode) {
    if (p.kind == BP_INTERVAL) {
        if (mode == MODE_GREATER) p.hi = 0xFFFFFFFFu;
        else if (mode == MODE_LESS) p.lo = 0u;
    }
    return p;
}

// block-wide min (MAX = false) / max of one value per thread (red: NTHREADS / 64 words); result
// in every thread
template <bool MAX>
__device__ __forceinline__ u32 block_minmax(u32 v, u32* red) {
    const int tid = cc_tid();
    v = wave_minmax_last<MAX>(v);
    __syncthreads();
    if ((tid & 63) == 63) red[tid >> 6] = v;
    __syncthreads();
    v = red[0];
#pragma unroll
    for (int w = 1; w < NTHREADS / 64; ++w) v = MAX ? max(v, red[w]) : min(v, red[w]);
    return v;
}

// k_spec's float4 input loads, non-temporal (the input is read once): C3 k_spec 3.09-3.11 ->
// 2.98-3.00 ms, C4 4.06 -> 3.97 ms on a fast-kind box (profiles/r05_ab_ntload.txt; CC_SPEC_NTLOAD=0
// for A/B)
#ifndef CC_SPEC_NTLOAD
#define CC_SPEC_NTLOAD 1
#endif
__device__ __forceinline__ float4 ld_in4(const float* p) {
#if CC_SPEC_NTLOAD
    typedef float v4f __attribute__((ext_vector_type(4)));
    const v4f v = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(p));
    return float4{v.x, v.y, v.z, v.w};
#else
    return *reinterpret_cast<const float4*>(p);
#endif
}

// k_sample's rows, non-temporal too (C3 k_sample 0.114 -> 0.055 ms; CC_SAMPLE_NT=0 for A/B).  The
// other read-once streams measured worse or equal that way (CC_RD_NT, A/B only: k_spec's mask
// 4.40 -> 4.89 ms at C4, k_seams' face planes 0.272 -> 0.285 ms, k_pass2's bit rows equal), and so
// did k_pass2's label stores (CC_P2_NTSTORE: 5.52 -> 5.80 ms): profiles/r05_ab_ntload.txt
#ifndef CC_SAMPLE_NT
#define CC_SAMPLE_NT 1
#endif
#ifndef CC_RD_NT
#define CC_RD_NT 0
#endif
#ifndef CC_P2_NTSTORE
#define CC_P2_NTSTORE 0
#endif
template <class T>
__device__ __forceinline__ T ld_once(const T* p) {
    if constexpr (CC_RD_NT) return __builtin_nontemporal_load(p);
    else return *p;
}
__device__ __forceinline__ float4 ld_sample4(const float* p) {
#if CC_SAMPLE_NT
    typedef float v4f __attribute__((ext_vector_type(4)));
    const v4f v = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(p));
    return float4{v.x, v.y, v.z, v.w};
#else
    return *reinterpret_cast<const float4*>(p);
#endif
}
__device__ __forceinline__ uint4 ld_once_u4(const void* p) {
#if CC_RD_NT
    typedef u32 v4u __attribute__((ext_vector_type(4)));
    const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
    return uint4{v.x, v.y, v.z, v.w};
#else
    return *reinterpret_cast<const uint4*>(p);
#endif
}

// k_sample: workgroup (b, part) reads every SAMPLE_PARTS-th sample row of block b and writes its
// (min, 0, max, 0); k_guess combines the parts of each block.
constexpr int SAMPLE_PARTS = 8;

// (the guess stays a launch of its own, k_guess: folding it in by a last-part-of-the-block count
// needed an agent-scope fence per workgroup -- an L2 write-back on gfx950 -- and measured k_sample
// 0.11 -> 0.25 ms at C3)
// The front's initial state, written by k_sample's threads before they sample (it replaced nine
// memsets of ~4 us each, then a launch of its own): ordered block min = ~0, max / NaN flag = 0,
// scalars, the k_fix count, seam overflow flags (+ their "any" flags at big[nb] / iovf[nt];
// fill = 1 sends everything to the global stitch), the inter-pair counts, the root segments and
// the scan's extra element.
// mflag / fchg (nullable, the device-gated k_fix of the one-read-back schedule): the seam marks
// and their list count (mflag[nt]) and the changed-faces flags, which the host-synchronised
// schedule clears only when the k_fix count it read back is non-zero.
// htab / hkeys + hpar (nullable, shards of the one-read-back schedule): the seam pair set and the
// seam map of the previous step cleared for this one (n_clear = the longest of all the ranges)
struct FrontClear {
    int64_t nb, nt;
    u32* smin; u32* smax_flag; u64* scalars; u32* FIX; u8* big; u8* iovf; u32* ipc; u32* seg; u32* rc_end;
    u8 fill;
    u32* mflag; u8* fchg;
    u64* htab; int64_t htab_n; u64* hkeys; u32* hpar; int64_t hm_n;
    u32* mlive;           // masked runs: the blocks' "any mask voxel" flags (k_mask_live), else null
    int64_t n_clear;      // the longest of the ranges (0: nothing to clear)
};
__device__ __forceinline__ void clear_front(const FrontClear& f, int64_t i) {
    if (f.htab && i < f.htab_n) f.htab[i] = ~0ull;
    if (f.hkeys && i < f.hm_n) { f.hkeys[i] = ~0ull; f.hpar[i] = (u32)i; }
    if (i < f.nb) f.smin[i] = 0xFFFFFFFFu;
    if (i < 2 * f.nb) { f.smax_flag[i] = 0u; f.seg[i] = 0u; }
    if (i <= f.nb) f.big[i] = f.fill;
    if (i <= f.nt) f.iovf[i] = f.fill;
    if (i < f.nt) f.ipc[i] = 0u;
    if (i < SCALARS) f.scalars[i] = 0ull;
    if (i == 0) { f.FIX[0] = 0u; f.rc_end[0] = 0u; }
    if (f.mflag && i <= f.nt) f.mflag[i] = 0u;
    if (f.fchg && i < f.nt) f.fchg[i] = 0;
    if (f.mlive && i < f.nb) f.mlive[i] = 0u;
}

// mask (nullable, masked runs): the part also reads the mask bytes of its sample rows and records
// whether one is set (q[1]); k_guess turns that into the block's live flag, so that k_mask_live
// scans only the blocks the sample found no mask voxel in
__global__ __launch_bounds__(NTHREADS) void k_sample(Geom g, const float* __restrict__ in, u32* part, FrontClear fc,
                                                     const u8* __restrict__ mask = nullptr) {
    __shared__ u32 red[NTHREADS / 64];
    for (int64_t i = (int64_t)blockIdx.x * NTHREADS + threadIdx.x; i < fc.n_clear; i += (int64_t)gridDim.x * NTHREADS)
        clear_front(fc, i);
    const int64_t b = blockIdx.x / SAMPLE_PARTS;
    const int pt = blockIdx.x % SAMPLE_PARTS;
    const int tid = cc_tid();
    int e0[3], el[3];
    block_extent(g, b, e0, el);
    const int nzs = max(1, el[0] / SAMPLE_DZ), nys = max(1, el[1] / SAMPLE_DY);
    const int zo = min(SAMPLE_DZ / 2, (el[0] - 1) / 2), yo = min(SAMPLE_DY / 2, (el[1] - 1) / 2);
    // SAMPLE_U rows of the part in flight per thread (one row at a time was latency-bound)
    constexpr int SAMPLE_U = 8;
    const int nrows = nzs * nys;
    auto sweep = [&](auto&& f) {
        for (int r0 = pt; r0 < nrows; r0 += SAMPLE_PARTS * SAMPLE_U)
            for (int x = tid; x < el[2]; x += NTHREADS) {
                float v[SAMPLE_U];
#pragma unroll
                for (int u = 0; u < SAMPLE_U; ++u) {
                    const int r = min(r0 + u * SAMPLE_PARTS, nrows - 1);    // repeats are harmless
                    const int z = e0[0] + (r / nys) * SAMPLE_DZ + zo, y = e0[1] + (r % nys) * SAMPLE_DY + yo;
                    v[u] = in[((int64_t)z * g.Y + y) * g.X + e0[2] + x];
                }
#pragma unroll
                for (int u = 0; u < SAMPLE_U; ++u) f(f2ord(__float_as_uint(v[u])));
            }
    };
    u32 mn = 0xFFFFFFFFu, mx = 0u;
    auto f = [&](u32 o) {
        mn = min(mn, o);
        mx = max(mx, o);
    };
    if (((g.X | e0[2] | el[2]) & 3) == 0) {
        // 16-B aligned rows: float4 per lane, 4 rows per workgroup pass, SAMPLE_U of them in
        // flight (the scalar walk waited on 8 dependent rounds of 8 rows per part)
        const int slot = tid >> 7, x4 = 4 * (tid & 127);
        const int nj = (nrows - pt + SAMPLE_PARTS - 1) / SAMPLE_PARTS;      // rows of this part
        for (int j0 = 0; j0 < nj; j0 += 4 * SAMPLE_U)
            for (int x = x4; x < el[2]; x += 512) {
                float4 v[SAMPLE_U];
#pragma unroll
                for (int u = 0; u < SAMPLE_U; ++u) {
                    const int j = min(j0 + 4 * u + slot, nj - 1);             // repeats are harmless
                    const int r = pt + SAMPLE_PARTS * j;
                    const int z = e0[0] + (r / nys) * SAMPLE_DZ + zo, y = e0[1] + (r % nys) * SAMPLE_DY + yo;
                    v[u] = ld_sample4(in + ((int64_t)z * g.Y + y) * g.X + e0[2] + x);
                }
#pragma unroll
                for (int u = 0; u < SAMPLE_U; ++u) {
                    f(f2ord(__float_as_uint(v[u].x))); f(f2ord(__float_as_uint(v[u].y)));
                    f(f2ord(__float_as_uint(v[u].z))); f(f2ord(__float_as_uint(v[u].w)));
                }
            }
    } else {
        sweep(f);
    }
    mn = block_minmax<false>(mn, red);
    mx = block_minmax<true>(mx, red);
    u32 mhit = 0;
    if (mask) {
        // every 4th of the part's sample rows, 16-B loads on aligned rows (a live region of any
        // size is met; the rest is k_mask_live's)
        bool hit = false;
        const bool a16 = ((g.X | e0[2] | el[2]) & 15) == 0;
        const int wpr = a16 ? el[2] / 16 : el[2];
        const int nr = (nrows - pt + 4 * SAMPLE_PARTS - 1) / (4 * SAMPLE_PARTS);
        for (int i = tid; i < nr * wpr; i += NTHREADS) {
            const int r = pt + 4 * SAMPLE_PARTS * (i / wpr), xi = i % wpr;
            const int z = e0[0] + (r / nys) * SAMPLE_DZ + zo, y = e0[1] + (r % nys) * SAMPLE_DY + yo;
            const u8* row = mask + ((int64_t)z * g.Y + y) * g.X + e0[2];
            if (a16) { const uint4 v = reinterpret_cast<const uint4*>(row)[xi]; hit |= (v.x | v.y | v.z | v.w) != 0u; }
            else hit |= row[xi] != 0;
        }
        mhit = __syncthreads_or(hit) ? 1u : 0u;
    }
    if (tid == 0) {
        u32* q = part + 4 * blockIdx.x;
        q[0] = mn; q[1] = mhit; q[2] = mx; q[3] = 0;
    }
}

// live (nullable, masked runs): a block whose sampled mask bytes hold a set one is live
__global__ void k_guess(int64_t nb, const u32* part, float thr, int mode, BlockParam* guess, u32* live = nullptr) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    const u32* q = part + 4 * SAMPLE_PARTS * b;
    u32 mn = 0xFFFFFFFFu, mx = 0u, mh = 0u;
    for (int p = 0; p < SAMPLE_PARTS; ++p) { mn = min(mn, q[4 * p]); mx = max(mx, q[4 * p + 2]); mh |= q[4 * p + 1]; }
    if (live) live[b] = mh ? 1u : 0u;
    const bool nan = mx > 0xFF800000u || mn < 0x007FFFFFu;
    // On continuous data the sampled extremes are not the block's, so the guessed bound misses
    // the exact one by a little: only tiles holding a voxel between the two are relabelled.
    guess[b] = widen(block_param(mn, mx, nan ? 1u : 0u, thr, mode), mode);
}

// Masked runs: live[b] = 1 iff block b holds a mask voxel.  The reference never reads a block whose
// mask is empty -- it returns 0 before reading the input (block_components.py:197-201) -- so such
// a block's tiles skip the front entirely (no input or mask read, no statistics: its labels are 0
// and its value 0 whatever its input holds).  One workgroup per (block, part): part p scans the
// block's rows p, p + LIVE_PARTS, ... from a part-dependent start (a live region is met within a
// few rows by most parts), and every workgroup stops once the block is known to be live; only
// blocks without a mask voxel are read whole (C4: 56 of 256 blocks, 0.94 GB of mask).
constexpr int LIVE_PARTS = 64;
constexpr int LIVE_THREADS = 256;
constexpr int LIVE_U = 4;        // loads in flight per thread and pass

__global__ __launch_bounds__(LIVE_THREADS) void k_mask_live(Geom g, const u8* __restrict__ mask, u32* live) {
    volatile u32* lv = live;
    {
        const int64_t b = blockIdx.x / LIVE_PARTS;
        const int p = (int)(blockIdx.x % LIVE_PARTS);
        if (__builtin_amdgcn_readfirstlane(lv[b])) return;
        int e0[3], el[3];
        block_extent(g, b, e0, el);
        const int nrows = el[0] * el[1];
        const int nmine = p < nrows ? (nrows - p + LIVE_PARTS - 1) / LIVE_PARTS : 0;   // rows p + LIVE_PARTS j
        if (nmine == 0) return;
        const int jstart = (int)((int64_t)nmine * p / LIVE_PARTS);                      // rotated start
        // item = 16, 4 or 1 mask bytes, as the rows' alignment allows
        const int isz = ((g.X | e0[2] | el[2]) & 15) == 0 ? 16 : ((g.X | e0[2] | el[2]) & 3) == 0 ? 4 : 1;
        const int wpr = el[2] / isz;                                                     // items per row
        const int per = LIVE_U * LIVE_THREADS;                                           // items per pass
        const int64_t total = (int64_t)nmine * wpr;
        for (int64_t i0 = 0, pass = 0; i0 < total; i0 += per, ++pass) {
            bool hit = false;
#pragma unroll
            for (int u = 0; u < LIVE_U; ++u) {
                const int64_t i = i0 + u * LIVE_THREADS + threadIdx.x;
                if (i < total) {
                    const int j = (int)((jstart + i / wpr) % nmine), r = p + LIVE_PARTS * j, xi = (int)(i % wpr);
                    const u8* row = mask + ((int64_t)(e0[0] + r / el[1]) * g.Y + e0[1] + r % el[1]) * g.X + e0[2];
                    if (isz == 16) { const uint4 v = reinterpret_cast<const uint4*>(row)[xi]; hit |= (v.x | v.y | v.z | v.w) != 0u; }
                    else if (isz == 4) hit |= reinterpret_cast<const u32*>(row)[xi] != 0u;
                    else hit |= row[xi] != 0;
                }
            }
            if (__syncthreads_or(hit)) {
                if (threadIdx.x == 0) lv[b] = 1u;
                break;
            }
            if ((pass & 1) == 1 && __builtin_amdgcn_readfirstlane(lv[b])) break;
        }
    }
}

struct SpecArgs {
    const BlockParam* guess;
    u32* smin; u32* smax; u32* sflag;
    u32* TB;                  // 4 per tile (see above)
    int64_t t0;               // first tile of this launch (the front runs in z-layer chunks)
    const u32* live = nullptr;   // masked runs: k_mask_live's flags (a block without one is skipped)
};

// workgroup b of n -> tile: the (b / 8)-th of the contiguous range of XCD b % 8 (workgroups are
// dealt to the 8 XCDs round-robin), so that x-neighbour tiles run on one XCD and a cache line
// they share (rows not 128-B aligned) meets in one L2 instead of being read / written by two.
// A bijection on [0, n).  Used when the rows are not line-aligned: C1 (X = 1250) k_spec 0.273 ->
// 0.257 ms, k_pass2 0.476 -> 0.437 ms (profiles/r04_ab_kspec.txt); on aligned rows the linear
// order stays (no gain there, round 3).
__device__ __forceinline__ int64_t xcd_contig(int64_t b, int64_t n) {
    const int64_t k = b & 7, i = b >> 3, q = n >> 3, r = n & 7;
    return k * q + (k < r ? k : r) + i;
}

// mask bytes: 4 per lane and plane (default), or 16 per lane staged through LDS (CC_MASK_STAGE=1,
// A/B only).  With plain input loads the staging won on the slow box kind (C4 k_spec<true>
// 4.90-4.95 -> 4.72-4.76 ms) and lost on the fast one (profiles/r05_ab_mstage*.txt); with the
// non-temporal input loads the 4-B loads win (fast kind 4.04-4.07 -> 3.96-3.97 ms:
// profiles/r05_ab_c4_order_mask.txt)
#ifndef CC_MASK_STAGE
#define CC_MASK_STAGE 0
#endif

// The front of k_spec for tile t: the tile's voxels in one read -> exact statistics (the
// block's atomics), the bit rows under the guessed interval [lo, hi] into L.rows, the tile's TB
// words.
// Returns whether the tile holds no foreground voxel (read off the statistics barrier).
template <bool HAS_MASK, int SIDES>
__device__ __forceinline__ bool spec_front(const Geom& g, const SpecArgs& sa, int64_t t, const TileInfo& ti,
                                           const float* __restrict__ in, const u8* __restrict__ mask, u32 lo,
                                           u32 hi, Pass1LDS& L, u32 (*red)[NTHREADS / 64]) {
    const int tid = cc_tid(), lane = tid & 63, wave = wave_id();
    // Statistics: ordered min / max of every voxel, and the nearest values around the guessed
    // bounds as the min / max of the wrapped distances k1 = o - lo and k2 = hi - o (mod 2^32) over
    // the used voxels: o - lo puts every voxel at or above lo below every voxel under it, so
    // min k1 gives the smallest value >= lo and max k1 the largest value < lo (hi - o likewise);
    // no per-voxel select on the side of the bound (TB is derived once per tile below).
    // The nearest values are taken over every voxel of the tile, masked or not: a superset of the
    // used voxels only moves them closer to the bounds, so k_params_verify can only send more tiles
    // to k_fix (a masked voxel between the guessed and the exact bound), never fewer -- and the
    // masked kernel saves the per-voxel selects (8 per float4).
    u32 mn = 0xFFFFFFFFu, mx = 0u, K1N = 0xFFFFFFFFu, K1X = 0u, K2N = 0xFFFFFFFFu, K2X = 0u;
    u64 myrow = 0;                                  // this thread's bit row (emptiness test)
    auto fgp = [&](u32 o) -> bool { return SIDES == 1 ? o >= lo : SIDES == 2 ? o <= hi : (o >= lo && o <= hi); };
    // one voxel (partial tiles)
    auto voxel = [&](float x, u32 mk) -> bool {
        const u32 o = f2ord(__float_as_uint(x));
        mn = min(mn, o);
        mx = max(mx, o);
        if (SIDES & 1) { const u32 k = o - lo; K1N = min(K1N, k); K1X = max(K1X, k); }
        if (SIDES & 2) { const u32 k = hi - o; K2N = min(K2N, k); K2X = max(K2X, k); }
        return (!HAS_MASK || mk != 0) && fgp(o);
    };
    // four voxels of one float4 (full tiles): the same, min / max folded three operands at a time
    // (returns the four ballots: the interval test and the mask test ballot separately and are
    // ANDed as lane masks -- a ballot of their combined bool went through a VGPR select and a
    // compare per value, 8 VALU per plane with a mask)
    auto quad = [&](float4 v, uchar4 mk, u64& b0, u64& b1, u64& b2, u64& b3) {
        const u32 o0 = f2ord(__float_as_uint(v.x)), o1 = f2ord(__float_as_uint(v.y));
        const u32 o2 = f2ord(__float_as_uint(v.z)), o3 = f2ord(__float_as_uint(v.w));
        mn = min(min(min(min(mn, o0), o1), o2), o3);
        mx = max(max(max(max(mx, o0), o1), o2), o3);
        if (SIDES & 1) {
            const u32 k0 = o0 - lo, k1 = o1 - lo, k2 = o2 - lo, k3 = o3 - lo;
            K1N = min(min(min(min(K1N, k0), k1), k2), k3);
            K1X = max(max(max(max(K1X, k0), k1), k2), k3);
        }
        if (SIDES & 2) {
            const u32 k0 = hi - o0, k1 = hi - o1, k2 = hi - o2, k3 = hi - o3;
            K2N = min(min(min(min(K2N, k0), k1), k2), k3);
            K2X = max(max(max(max(K2X, k0), k1), k2), k3);
        }
        b0 = __ballot(fgp(o0)); b1 = __ballot(fgp(o1)); b2 = __ballot(fgp(o2)); b3 = __ballot(fgp(o3));
        if (HAS_MASK) {
            b0 &= __ballot(mk.x != 0); b1 &= __ballot(mk.y != 0);
            b2 &= __ballot(mk.z != 0); b3 &= __ballot(mk.w != 0);
        }
    };
    const bool f4 = ti.lz == TZ && ti.ly == TY && ti.lx == TX && ((ti.x0 | (int)(g.X & 3)) & 3) == 0;
    if (f4) {
        // Full, 16-B aligned tile: float4 per lane (4 rows of 64 voxels per load instruction, a
        // quarter of the load instructions of the lane = x walk).  Wave w owns rows y = 4w .. 4w+3
        // of every plane; lane l holds x = 4 (l % 16) .. + 3 of row 4w + l / 16.  The four
        // ballots of plane z (value j of every lane) are parked in lane z, then each lane m
        // assembles tile row (z = m / 4, y = 4w + m % 4) in the split form from them.
        const int i4 = 4 * (lane & 15);
        const int64_t sz = g.Y * g.X;
        const float* pz = in + ((int64_t)ti.z0 * g.Y + ti.y0 + 4 * wave + (lane >> 4)) * g.X + ti.x0 + i4;
#if !CC_MASK_STAGE
        const u8* mz = HAS_MASK ? mask + (pz - in) : nullptr;
#else
        // mask bytes 16 per lane: per group of 4 planes lane L loads 16 B of
        // plane z0 + L / 16, row 4w + (L / 4) % 4, x = 16 (L % 4) and stages them in the wave's
        // 1 KB of LDS (L.key, unused until the tile CCL), where lane m finds its 4 bytes of plane a
        // at word a * 64 + m (one 16-B load instead of four 4-B loads per lane and group)
        const u8* mz16 = HAS_MASK ? mask + ((int64_t)ti.z0 * g.Y + ti.y0 + 4 * wave + ((lane >> 2) & 3)) * g.X + ti.x0 +
                                        16 * (lane & 3) + (int64_t)(lane >> 4) * sz
                                  : nullptr;
        u32* mstage = L.key + wave * 256;
#endif
        constexpr int RZ4 = 4;
        u32 R[8] = {0, 0, 0, 0, 0, 0, 0, 0};      // lane z: ballots (lo, hi) of values 0..3 of plane z
        auto plane_bits = [&](int z, float4 v, uchar4 mk) {
            u64 b0, b1, b2, b3;
            quad(v, mk, b0, b1, b2, b3);
            CC_WRITELANE2(R[0], R[1], (u32)b0, (u32)(b0 >> 32), z);
            CC_WRITELANE2(R[2], R[3], (u32)b1, (u32)(b1 >> 32), z);
            CC_WRITELANE2(R[4], R[5], (u32)b2, (u32)(b2 >> 32), z);
            CC_WRITELANE2(R[6], R[7], (u32)b3, (u32)(b3 >> 32), z);
        };
#pragma unroll
        for (int z0 = 0; z0 < TZ; z0 += RZ4) {
            float4 v[RZ4];
            uchar4 mk[RZ4];
#if CC_MASK_STAGE
            if (HAS_MASK) reinterpret_cast<uint4*>(mstage)[lane] = ld_once_u4(mz16 + z0 * sz);
            auto ld = [&](int a) {
                v[a] = ld_in4(pz + (z0 + a) * sz);
                if (HAS_MASK) mk[a] = __builtin_bit_cast(uchar4, mstage[a * 64 + lane]);
            };
#else
            auto ld = [&](int a) {
                v[a] = ld_in4(pz + (z0 + a) * sz);
                if (HAS_MASK) mk[a] = *reinterpret_cast<const uchar4*>(mz + (z0 + a) * sz);
            };
#endif
#pragma unroll
            for (int a = 0; a < RZ4; ++a) {
                // each load issued right before its use, one in flight per wave (an empty asm
                // with a memory clobber keeps the next load below the previous processing).  More
                // in flight measured slower on large volumes -- two or four register loads, and a
                // ring of four 1-KB LDS-DMA slots per wave (C3 k_spec 3.69 -> 3.87 ms, C4 masked
                // 4.89 -> 5.27 ms; only C2 gained, 0.179 -> 0.172 ms): DESIGN.md §3
                asm volatile("" ::: "memory");
                ld(a);
                plane_bits(z0 + a, v[a], HAS_MASK ? mk[a] : uchar4{});
            }
        }
        // row m = 4 z + q: bits 16 q .. 16 q + 15 of ballot j are voxels x = 4 i + j, i = 0..15
        const int zz = lane >> 2, qq = lane & 3;
        u32 seg[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const u32 blo = (u32)__shfl((int)R[2 * j], zz, 64), bhi = (u32)__shfl((int)R[2 * j + 1], zz, 64);
            seg[j] = ((qq < 2 ? blo : bhi) >> (16 * (qq & 1))) & 0xFFFFu;
        }
        // split form: even voxels x = 4i (j = 0), 4i + 2 (j = 2) -> bits 2i, 2i + 1 of the low half
        const u32 even = spread2(seg[0]) | (spread2(seg[2]) << 1), odd = spread2(seg[1]) | (spread2(seg[3]) << 1);
        myrow = ((u64)odd << 32) | even;
        L.rows[zz * TY + 4 * wave + qq] = myrow;
    } else {
        for (int i = tid; i < NROWS; i += NTHREADS) L.rows[i] = 0;
        __syncthreads();
        const u64 lanes = ti.lx >= 64 ? ~0ull : ((1ull << ti.lx) - 1);
        u32 mlo = 0, mhi = 0;                     // lane j: row mask of slot j (see load_rows)
        for_tile_rows<HAS_MASK>(g, ti, in, mask, [&](int j, float x, u32 mk) {
            const u64 bal = __ballot(voxel(x, mk)) & lanes;
            const u32 blo = (u32)bal, bhi = (u32)(bal >> 32);
            CC_WRITELANE2(mlo, mhi, blo, bhi, j);
        });
        const int r = slot_row(lane, wave);
        if (r / TY < ti.lz && r % TY < ti.ly) {
            myrow = split_row(((u64)mhi << 32) | mlo);
            L.rows[r] = myrow;
        }
    }
    const u32 nzw = __ballot(myrow != 0) ? 1u : 0u;
    mn = wave_min(mn);
    mx = wave_max(mx);
    if (SIDES & 1) { K1N = wave_min(K1N); K1X = wave_max(K1X); }
    if (SIDES & 2) { K2N = wave_min(K2N); K2X = wave_max(K2X); }
    if (lane == 0) {
        red[0][wave] = mn; red[1][wave] = mx; red[2][wave] = K1N; red[3][wave] = K1X; red[4][wave] = K2N;
        red[5][wave] = K2X; red[6][wave] = nzw;
    }
    __syncthreads();
    u32 nz = 0;
#pragma unroll
    for (int w = 0; w < NTHREADS / 64; ++w) nz |= red[6][w];
    if (tid == 0) {
        for (int w = 1; w < NTHREADS / 64; ++w) {
            mn = min(mn, red[0][w]); mx = max(mx, red[1][w]);
            K1N = min(K1N, red[2][w]); K1X = max(K1X, red[3][w]); K2N = min(K2N, red[4][w]); K2X = max(K2X, red[5][w]);
        }
        atomicMin(sa.smin + ti.block, mn);
        atomicMax(sa.smax + ti.block, mx);
        if (mx > 0xFF800000u || mn < 0x007FFFFFu) atomicOr(sa.sflag + ti.block, 1u);    // NaN
        // TB from the wrapped distances: A = max used o < lo, B = min used o >= lo, C = max used
        // o <= hi, D = min used o > hi (0 / ~0 when there is none)
        {
            u32 A = 0u, B = 0xFFFFFFFFu, C = 0u, D = 0xFFFFFFFFu;
            if (SIDES & 1) {
                if ((u64)K1N + lo < (1ull << 32)) B = K1N + lo;
                if ((u64)K1X + lo >= (1ull << 32)) A = K1X + lo;
            }
            if (SIDES & 2) {
                if (K2N <= hi) C = hi - K2N;
                if (K2X > hi) D = hi - K2X;
            }
            u32* tb = sa.TB + 4 * t;
            tb[0] = A; tb[1] = B; tb[2] = C; tb[3] = D;
        }
    }
    return nz == 0;
}

// timing probe of the clock tool (tools/clock_probe.hip defines it: per-workgroup core / wall
// clock stamps in k_spec and k_pass2); empty in the library
#ifndef CC_KERNEL_PROBE
#define CC_KERNEL_PROBE
#define CC_KERNEL_PROBE_END
#endif

// SIDES: bounds of the guessed interval that can move (1 lower: 'greater', 2 upper: 'less', 3 both)
// ABL (kernel ablation harness tools/ablate.hip only; 0 in the library): 99 stop once the bit rows
// are in LDS (loads, ballots, statistics), else as pass1_finish's ABL
template <bool HAS_MASK, int SIDES, int ABL = 0>
__global__ __launch_bounds__(NTHREADS) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_spec(
    Geom g, SpecArgs sa, const float* __restrict__ in, const u8* __restrict__ mask, u64* BITS, face_t* FACES,
    u32* COUNT, u32* P, u64* KEY) {
    CC_KERNEL_PROBE
    __shared__ Pass1LDS L;
    __shared__ u32 red[7][NTHREADS / 64];
    const int64_t t = sa.t0 + ((g.X & 31) ? xcd_contig(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x);
    const TileInfo ti = tile_info(g, t);
    if (HAS_MASK && sa.live && !__builtin_amdgcn_readfirstlane(sa.live[ti.block])) {
        // a block without a mask voxel: nothing is read, the tile is empty (COUNT 0, zero faces)
        pass1_finish<ABL % 99>(g, t, ti, BITS, FACES, COUNT, P, KEY, L, true, nullptr, 1);
        return;
    }
    const BlockParam p = uniform_bp(sa.guess[ti.block]);
    if (p.kind != BP_INTERVAL) {                   // no guess: statistics only, k_fix labels the tile
        stats_tile(g, ti, in, sa.smin, sa.smax, sa.sflag, red);
        return;
    }
    const bool empty = spec_front<HAS_MASK, SIDES>(g, sa, t, ti, in, mask, p.lo, p.hi, L, red);
    if (ABL == 99) return;
    pass1_finish<ABL % 99>(g, t, ti, BITS, FACES, COUNT, P, KEY, L, true, nullptr, empty ? 1 : 0);
    CC_KERNEL_PROBE_END
}

// are the bits computed with the guess G those of the exact parameters T? (see above)
__device__ __forceinline__ bool spec_valid(const BlockParam& G, BlockParam T, const u32* tb, int mode) {
    if (G.kind != BP_INTERVAL || T.kind != BP_INTERVAL) return false;
    T = widen(T, mode);
    if (T.lo != G.lo && (T.lo > G.lo ? tb[1] < T.lo : tb[0] >= T.lo)) return false;
    if (T.hi != G.hi && (T.hi < G.hi ? tb[2] > T.hi : tb[3] <= T.hi)) return false;
    return true;
}

// FIX[0] = number of tiles to relabel, FIX[1..] = their ids
__global__ void k_verify(Geom g, const BlockParam* guess, const BlockParam* bp, const u32* TB, int mode, u32* FIX) {
    CC_FOR(t, g.n_tiles) {
        const int64_t b = tile_info(g, t).block;
        if (!spec_valid(guess[b], bp[b], TB + 4 * t, mode)) FIX[1 + atomicAdd(FIX, 1u)] = (u32)t;
    }
}

// k_block_params and k_verify in one launch: every tile derives its block's exact parameters from
// the statistics (a few dozen float ops), the block's first tile stores them for k_fix
// live (nullable, masked runs): a block without a mask voxel gets no foreground (BP_EMPTY) and
// none of its tiles is listed (k_spec left them empty without reading them)
__global__ void k_params_verify(Geom g, const BlockParam* guess, const u32* smin, const u32* smax, const u32* sflag,
                                float thr, int mode, BlockParam* bp, const u32* TB, u32* FIX, const u32* live) {
    CC_FOR(t, g.n_tiles) {
        const TileInfo ti = tile_info(g, t);
        const int64_t b = ti.block;
        const bool dead = live && !live[b];
        BlockParam T;
        if (dead) { T.kind = BP_EMPTY; T.lo = 1; T.hi = 0; T.pad = 0; T.mn = 0.0f; T.m = 0.0f; }
        else T = block_param(smin[b], smax[b], sflag[b], thr, mode);
        const bool first = (ti.iz == 0 || g.tblk[0][ti.iz - 1] != g.tblk[0][ti.iz]) &&
                           (ti.iy == 0 || g.tblk[1][ti.iy - 1] != g.tblk[1][ti.iy]) &&
                           (ti.ix == 0 || g.tblk[2][ti.ix - 1] != g.tblk[2][ti.ix]);
        if (first) bp[b] = T;
        if (!dead && !spec_valid(guess[b], T, TB + 4 * t, mode)) FIX[1 + atomicAdd(FIX, 1u)] = (u32)t;
    }
}

// the 14 tiles whose seams read the faces of tile f (f itself and the 13 that have it as a
// lex-negative neighbour): d = 0 .. 13, each marked once (flag) and listed in LIST[1 .. LIST[0]]
__device__ __forceinline__ void mark_seam(const Geom& g, u32 f, u32 d, u32* flag, u32* LIST) {
    const TileInfo ti = tile_info(g, f);
    int dz = 0, dy = 0, dx = 0;
    if (d > 0) {
        const int c = (int)d - 1;               // 0..12: (0,0,1), (0,1,-1..1), (1,-1..1,-1..1)
        if (c == 0) { dx = 1; }
        else if (c < 4) { dy = 1; dx = c - 2; }
        else { dz = 1; dy = (c - 4) / 3 - 1; dx = (c - 4) % 3 - 1; }
    }
    const int iz = ti.iz + dz, iy = ti.iy + dy, ix = ti.ix + dx;
    if (iz >= g.nt[0] || iy < 0 || iy >= g.nt[1] || ix < 0 || ix >= g.nt[2]) return;
    const u32 t = (u32)(((int64_t)iz * g.nt[1] + iy) * g.nt[2] + ix);
    if (atomicExch(&flag[t], 1u) == 0u) LIST[1 + atomicAdd(LIST, 1u)] = t;
}

// k_fix: pass 1 with the exact parameters for the tiles listed in FIX[1 .. FIX[0]] (k_params_verify),
// and a tile whose faces changed marks the seams to redo (flag / LIST for k_seams).  fchg[t] = 1
// when the tile's faces changed; tiles k_spec only read for statistics (no guess) hold no faces
// from this run and are always flagged.  The grid walks the list: the one-read-back schedule
// launches a fixed grid without reading the count (with nothing to fix every workgroup reads one
// word and leaves), the host-synchronised one a workgroup per listed tile.  fchg, flag and
// LIST[0] are cleared before (the front clear in k_sample / memsets).  fchg = flag = nullptr: no
// seams to mark (the one-read-back schedule runs k_seams after k_fix).
// (no waves-per-EU bound: under the 64-VGPR bound of k_fix the loop spilled; this kernel sees
// ~1 % of the tiles on continuous input and none on quantized input)
template <bool HAS_MASK>
__global__ __launch_bounds__(NTHREADS) void k_fix_dev(
    Geom g, const u32* FIX, const BlockParam* bp, const BlockParam* guess, const float* __restrict__ in,
    const u8* __restrict__ mask, float thr, int mode, u64* BITS, face_t* FACES, u32* COUNT, u32* P, u64* KEY,
    u8* fchg, u32* flag, u32* LIST) {
    __shared__ Pass1LDS L;
    const u32 n = __builtin_amdgcn_readfirstlane(FIX[0]);
#pragma nounroll
    for (u32 i = blockIdx.x; i < n; i += gridDim.x) {
        const int64_t t = __builtin_amdgcn_readfirstlane(FIX[1 + i]);
        const TileInfo ti = uniform_ti(tile_info(g, t));
        const BlockParam p = uniform_bp(bp[ti.block]);
        const bool fresh = __builtin_amdgcn_readfirstlane(guess[ti.block].kind) == BP_INTERVAL;
        if (fchg && !fresh && cc_tid() == 0) fchg[t] = 1;
        pass1_tile<HAS_MASK>(g, t, ti, p, in, mask, thr, mode, BITS, FACES, COUNT, P, KEY, L, true,
                             fresh ? fchg : nullptr);
        __syncthreads();                              // fchg[t] (thread 0) visible to the workgroup
        if (flag && cc_tid() < 14 && fchg[t]) mark_seam(g, (u32)t, (u32)cc_tid(), flag, LIST);
        __syncthreads();                              // L is reused by the next tile
    }
}

// ------------------------------------------------------------------------------------------
// k_stitch<INTER>: unions across tile seams.
//   INTER = false: seams inside one block, 26-connectivity (13 tile directions).
//   INTER = true : seams on block faces, 6-connectivity (3 face directions).
// Keys: first-voxel index (intra) or rid (inter); the union keeps the smaller key as root.
// ------------------------------------------------------------------------------------------
// Stage the face planes tile t needs from its three face neighbours into LDS, in the FACE_STRIDE
// layout: own ZLO/YLO/XLO and the z-/y-/x-lower neighbours' ZHI/YHI/XHI (0 where absent).  One
// parallel load round instead of dependent global loads per face cube.
// ST: u32 (k_stitch) or face_t (k_seams: half the LDS, twice the waves per CU)
template <class ST>
__device__ __forceinline__ void stage_faces(const Geom& g, const face_t* __restrict__ FACES, int64_t t,
                                            const TileInfo& ti, ST* S, int tid, int nthr) {
    const int64_t sz = (int64_t)g.nt[1] * g.nt[2], sy = g.nt[2];
    // source tile of entry i: own lower faces, the lower neighbours' upper faces (-1: absent)
    auto src = [&](int i) -> int64_t {
        if (i < F_ZHI || (i >= F_YLO && i < F_YHI) || (i >= F_XLO && i < F_XHI)) return t;
        if (i < F_YLO) return ti.iz > 0 ? t - sz : -1;
        if (i < F_XLO) return ti.iy > 0 ? t - sy : -1;
        return ti.ix > 0 ? t - 1 : -1;
    };
    if (nthr == 64) {
        // one wave: every load issued before the first LDS write (one memory round trip), two
        // 16-bit entries per lane and load; the face regions are multiples of 128 entries, so
        // each unrolled step reads one tile
        constexpr int NJ = (FACE_STRIDE / 2 + 63) / 64;
        static_assert(F_Z % 128 == 0 && F_Y % 128 == 0 && F_X % 128 == 0, "face regions are whole waves");
        const u32* FW = (const u32*)FACES;
        u32 v[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int w = tid + 64 * j;
            const int64_t ts = src(128 * j);
            v[j] = (w < FACE_STRIDE / 2 && ts >= 0) ? ld_once(FW + ts * (FACE_STRIDE / 2) + w) : 0u;
        }
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int w = tid + 64 * j;
            if (w < FACE_STRIDE / 2) {
                if constexpr (sizeof(ST) == 2) ((u32*)S)[w] = v[j];      // the two entries as stored
                else { S[2 * w] = v[j] & 0xFFFFu; S[2 * w + 1] = v[j] >> 16; }
            }
        }
        return;
    }
    for (int i = tid; i < FACE_STRIDE; i += nthr) {
        const int64_t ts = src(i);
        S[i] = ts >= 0 ? (ST)FACES[ts * FACE_STRIDE + i] : (ST)0;
    }
}

// Up to two distinct neighbour components of one face cube, gathered without branches; a third
// distinct one sets ovf and the caller falls back to visiting every neighbour.
struct Cand {
    u32 b1 = 0, b2 = 0;
    bool ovf = false;
    __device__ __forceinline__ void add(u32 b) {
        const bool new1 = b && b1 && ((b ^ b1) & FK_MASK);
        const bool new2 = new1 && b2 && ((b ^ b2) & FK_MASK);
        ovf |= new2;
        b2 = (new1 && !b2) ? b : b2;
        b1 = b1 ? b1 : b;
    }
};

// Connected neighbour entry or 0: face cube a (bits ab) and neighbour entry b with the 4-bit face
// selections sa (own side) and sb (neighbour side).
__device__ __forceinline__ u32 face_link(u32 ab, u32 sa, u32 b, u32 sb) {
    return ((ab & sa) && ((b >> FK_BITS) & sb)) ? b : 0u;
}

// 3x3 neighbourhood across a face plane: own entry a at (p, q), neighbour plane FN with row
// stride QS and valid extent np x nq.  Calls U(t, a, tn, b) once per distinct neighbour component.
template <int QS, class UF>
__device__ __forceinline__ void face3x3(const u32* FN, u32 a, int p, int q, int np, int nq, int64_t t, int64_t tn,
                                        UF& U) {
    const u32 ab = a >> FK_BITS;
    auto nb = [&](int dp, int dq) -> u32 {
        const int pp = p + dp, qq = q + dq;
        const bool ok = pp >= 0 && pp < np && qq >= 0 && qq < nq;
        const u32 b = FN[ok ? pp * QS + qq : 0];
        return ok ? face_link(ab, fsel(self_sel(dp), self_sel(dq)), b, fsel(nbr_sel(dp), nbr_sel(dq))) : 0u;
    };
    Cand c;
#pragma unroll
    for (int dp = -1; dp <= 1; ++dp)
#pragma unroll
        for (int dq = -1; dq <= 1; ++dq) c.add(nb(dp, dq));
    if (c.b1) U(t, a, tn, c.b1);
    if (c.b2) U(t, a, tn, c.b2);
    if (c.ovf) {
#pragma unroll 1
        for (int i = 0; i < 9; ++i) {
            const u32 b = nb(i / 3 - 1, i % 3 - 1);
            if (b) U(t, a, tn, b);
        }
    }
}

// Three neighbours along one axis of an edge: own entry a at q, neighbour row FR (stride 1 in q)
// of extent nq; sa/sb fixed selection of the other axis (own / neighbour side).
template <bool Q_IS_P, class UF>
__device__ __forceinline__ void edge3(const face_t* FR, int RS, u32 a, int q, int nq, int so, int sn, int64_t t,
                                      int64_t te, UF& U) {
    const u32 ab = a >> FK_BITS;
    Cand c;
#pragma unroll
    for (int d = -1; d <= 1; ++d) {
        const int qq = q + d;
        const bool ok = qq >= 0 && qq < nq;
        const u32 b = FR[(ok ? qq : 0) * RS];
        const u32 sa = Q_IS_P ? fsel(self_sel(d), so) : fsel(so, self_sel(d));
        const u32 sb = Q_IS_P ? fsel(nbr_sel(d), sn) : fsel(sn, nbr_sel(d));
        c.add(ok ? face_link(ab, sa, b, sb) : 0u);
    }
    if (c.b1) U(t, a, te, c.b1);
    if (c.b2) U(t, a, te, c.b2);
    if (c.ovf) {
#pragma unroll 1
        for (int d = -1; d <= 1; ++d) {
            const int qq = q + d;
            if (qq < 0 || qq >= nq) continue;
            const u32 sa = Q_IS_P ? fsel(self_sel(d), so) : fsel(so, self_sel(d));
            const u32 sb = Q_IS_P ? fsel(nbr_sel(d), sn) : fsel(sn, nbr_sel(d));
            const u32 b = face_link(ab, sa, FR[qq * RS], sb);
            if (b) U(t, a, te, b);
        }
    }
}

// Unions across the lower seams of tile t: calls U(t, entry, t_nbr, entry_nbr) for connected face
// cubes (face entry = k | bits << FK_BITS), at least once per connected pair of tile components.
// S = stage_faces() copy; edge and corner neighbours are read from FACES.
//   INTER = false: seams inside one block, 26-connectivity (13 tile directions).
//   INTER = true : seams on block faces, 6-connectivity (3 face directions).
template <bool INTER, class UF, bool EDGES_ONLY = false>
__device__ __forceinline__ void stitch_tile(const Geom& g, const face_t* __restrict__ FACES, const u32* S,
                                            int64_t t, const TileInfo& ti, int tid, int nthr, UF&& U) {
    const int ncy = (ti.ly + 1) / 2, ncx = (ti.lx + 1) / 2, ncz = (ti.lz + 1) / 2;
    const int64_t sz = (int64_t)g.nt[1] * g.nt[2], sy = g.nt[2];

    // ---------------- z-lower seam ----------------
    if (ti.iz > 0) {
        const bool same_z = g.tblk[0][ti.iz] == g.tblk[0][ti.iz - 1];
        const int64_t tn = t - sz;
        if (INTER) {
            if (!same_z)
                for (int e = tid; e < ncy * CX; e += nthr) {
                    const int cx = e % CX;
                    if (cx >= ncx) continue;
                    const u32 a = S[F_ZLO + e];
                    if (!a) continue;
                    const u32 b = S[F_ZHI + e];
                    if ((a >> FK_BITS) & (b >> FK_BITS)) U(t, a, tn, b);
                }
        } else if (same_z) {
            if (!EDGES_ONLY)
            for (int e = tid; e < ncy * CX; e += nthr) {          // face (-1, 0, 0): offsets (dy, dx)
                const int cy = e / CX, cx = e % CX;
                if (cx >= ncx) continue;
                const u32 a = S[F_ZLO + e];
                if (a) face3x3<CX>(S + F_ZHI, a, cy, cx, ncy, ncx, t, tn, U);
            }
            for (int s = -1; s <= 1; s += 2) {                    // edges (-1, s, 0)
                const int jy = ti.iy + s;
                if (jy < 0 || jy >= g.nt[1] || g.tblk[1][jy] != g.tblk[1][ti.iy]) continue;
                const int64_t te = tn + s * sy;
                const int lyn = g.tlen[1][jy];
                const int cyo = s < 0 ? 0 : ncy - 1, cyn = s < 0 ? (lyn - 1) / 2 : 0;
                const int jo = s < 0 ? 0 : (ti.ly - 1) & 1, jn = s < 0 ? (lyn - 1) & 1 : 0;
                const face_t* FR = FACES + te * FACE_STRIDE + F_ZHI + cyn * CX;
                for (int cx = tid; cx < ncx; cx += nthr) {
                    const u32 a = S[F_ZLO + cyo * CX + cx];
                    if (a) edge3<false>(FR, 1, a, cx, ncx, jo, jn, t, te, U);
                }
            }
            for (int s = -1; s <= 1; s += 2) {                    // edges (-1, 0, s)
                const int jx = ti.ix + s;
                if (jx < 0 || jx >= g.nt[2] || g.tblk[2][jx] != g.tblk[2][ti.ix]) continue;
                const int64_t te = tn + s;
                const int lxn = g.tlen[2][jx];
                const int cxo = s < 0 ? 0 : ncx - 1, cxn = s < 0 ? (lxn - 1) / 2 : 0;
                const int io = s < 0 ? 0 : (ti.lx - 1) & 1, in_ = s < 0 ? (lxn - 1) & 1 : 0;
                const face_t* FR = FACES + te * FACE_STRIDE + F_ZHI + cxn;
                for (int cy = tid; cy < ncy; cy += nthr) {
                    const u32 a = S[F_ZLO + cy * CX + cxo];
                    if (a) edge3<true>(FR, CX, a, cy, ncy, io, in_, t, te, U);
                }
            }
            if (tid < 4) {                                         // corners (-1, s1, s2)
                const int s1 = (tid & 2) ? 1 : -1, s2 = (tid & 1) ? 1 : -1;
                const int jy = ti.iy + s1, jx = ti.ix + s2;
                if (jy >= 0 && jy < g.nt[1] && jx >= 0 && jx < g.nt[2] &&
                    g.tblk[1][jy] == g.tblk[1][ti.iy] && g.tblk[2][jx] == g.tblk[2][ti.ix]) {
                    const int64_t tc = tn + s1 * sy + s2;
                    const int lyn = g.tlen[1][jy], lxn = g.tlen[2][jx];
                    const int cyo = s1 < 0 ? 0 : ncy - 1, cyn = s1 < 0 ? (lyn - 1) / 2 : 0;
                    const int cxo = s2 < 0 ? 0 : ncx - 1, cxn = s2 < 0 ? (lxn - 1) / 2 : 0;
                    const int jo = s1 < 0 ? 0 : (ti.ly - 1) & 1, jn = s1 < 0 ? (lyn - 1) & 1 : 0;
                    const int io = s2 < 0 ? 0 : (ti.lx - 1) & 1, in_ = s2 < 0 ? (lxn - 1) & 1 : 0;
                    const u32 a = S[F_ZLO + cyo * CX + cxo];
                    const u32 b = FACES[tc * FACE_STRIDE + F_ZHI + cyn * CX + cxn];
                    if (a && b && ((a >> FK_BITS) & fsel(jo, io)) && ((b >> FK_BITS) & fsel(jn, in_)))
                        U(t, a, tc, b);
                }
            }
        }
    }
    // ---------------- y-lower seam ----------------
    if (ti.iy > 0) {
        const bool same_y = g.tblk[1][ti.iy] == g.tblk[1][ti.iy - 1];
        const int64_t tn = t - sy;
        if (INTER) {
            if (!same_y)
                for (int e = tid; e < ncz * CX; e += nthr) {
                    const int cx = e % CX;
                    if (cx >= ncx) continue;
                    const u32 a = S[F_YLO + e];
                    if (!a) continue;
                    const u32 b = S[F_YHI + e];
                    if ((a >> FK_BITS) & (b >> FK_BITS)) U(t, a, tn, b);
                }
        } else if (same_y) {
            if (!EDGES_ONLY)
            for (int e = tid; e < ncz * CX; e += nthr) {          // face (0, -1, 0): offsets (dz, dx)
                const int cz = e / CX, cx = e % CX;
                if (cx >= ncx) continue;
                const u32 a = S[F_YLO + e];
                if (a) face3x3<CX>(S + F_YHI, a, cz, cx, ncz, ncx, t, tn, U);
            }
            for (int s = -1; s <= 1; s += 2) {                    // edges (0, -1, s)
                const int jx = ti.ix + s;
                if (jx < 0 || jx >= g.nt[2] || g.tblk[2][jx] != g.tblk[2][ti.ix]) continue;
                const int64_t te = tn + s;
                const int lxn = g.tlen[2][jx];
                const int cxo = s < 0 ? 0 : ncx - 1, cxn = s < 0 ? (lxn - 1) / 2 : 0;
                const int io = s < 0 ? 0 : (ti.lx - 1) & 1, in_ = s < 0 ? (lxn - 1) & 1 : 0;
                const face_t* FR = FACES + te * FACE_STRIDE + F_YHI + cxn;
                for (int cz = tid; cz < ncz; cz += nthr) {
                    const u32 a = S[F_YLO + cz * CX + cxo];
                    if (a) edge3<true>(FR, CX, a, cz, ncz, io, in_, t, te, U);
                }
            }
        }
    }
    // ---------------- x-lower seam ----------------
    if (ti.ix > 0) {
        const bool same_x = g.tblk[2][ti.ix] == g.tblk[2][ti.ix - 1];
        const int64_t tn = t - 1;
        if (INTER) {
            if (!same_x)
                for (int e = tid; e < ncz * CY; e += nthr) {
                    const int cy = e % CY;
                    if (cy >= ncy) continue;
                    const u32 a = S[F_XLO + e];
                    if (!a) continue;
                    const u32 b = S[F_XHI + e];
                    if ((a >> FK_BITS) & (b >> FK_BITS)) U(t, a, tn, b);
                }
        } else if (same_x && !EDGES_ONLY) {
            for (int e = tid; e < ncz * CY; e += nthr) {          // face (0, 0, -1): offsets (dz, dy)
                const int cz = e / CY, cy = e % CY;
                if (cy >= ncy) continue;
                const u32 a = S[F_XLO + e];
                if (a) face3x3<CY>(S + F_XHI, a, cz, cy, ncz, ncy, t, tn, U);
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// Intra-block seams without global atomics, in two launches:
//   k_seams         one wave per tile: connected (own component, neighbour component) pairs
//                   across its lower intra-block seams, deduplicated in LDS, appended to the
//                   tile's slot list as block-local ids (local tile << 12 | k);
//   k_block_uf      one workgroup per block: union-find over the block's components in LDS fed
//                   by those lists, roots = smallest first voxel; the result goes to P.
// A block whose lists overflow, or with more than SB_MAXT tiles or SB_LCAP components, is
// flagged in big[] and stitched by k_stitch<false> instead.
// ------------------------------------------------------------------------------------------
constexpr int TPC = 512;           // pair slots per tile
constexpr int SB_THREADS = 1024;
constexpr int SB_MAXT = 1024;
constexpr int SB_LCAP = 8192;

// index of tile t inside its block (z-major over the block's tiles); tile ids fit u32
__device__ __forceinline__ u32 block_local(const Geom& g, u32 t) {
    const u32 n2 = (u32)g.nt[2], n1 = (u32)g.nt[1];
    const u32 q = t / n2, ix = t - q * n2, iz = q / n1, iy = q - iz * n1;
    const int bz = g.tblk[0][iz], by = g.tblk[1][iy], bx = g.tblk[2][ix];
    return (u32)(((iz - g.bt0[0][bz]) * g.btn[1][by] + (iy - g.bt0[1][by])) * g.btn[2][bx] + (ix - g.bt0[2][bx]));
}

// Wave-level duplicate filter: lanes whose key equals the first active lane's key drop out (two
// rounds); returns whether this lane still has to emit its key.
__device__ __forceinline__ bool wave_first(u64 key) {
    const u32 lane = __lane_id();
#pragma unroll 1
    for (int r = 0; r < 2; ++r) {
        const u64 lk = ((u64)__builtin_amdgcn_readfirstlane((u32)(key >> 32)) << 32) |
                       (u64)__builtin_amdgcn_readfirstlane((u32)key);
        const u32 leader = __builtin_amdgcn_readfirstlane(lane);
        if (key == lk) return lane == leader;
    }
    return true;
}

constexpr int SP_WAVES = 4;            // waves (tiles) per workgroup of the seam kernels

// ------------------------------------------------------------------------------------------
// k_seams: the tile's three lower seams with voxel-row bit masks, one wave per tile.
//
// A seam plane is rebuilt from the staged face entries as rows of bits (z seam: rows y, bits x;
// y seam: rows z, bits x; x seam: rows z, bits y); lane r holds row r of both sides.  Voxel x of
// own row r touches voxel x + dx of neighbour row r + dr; C = A & shift(B, dx) marks those, and
// one pair is emitted per run of C (consecutive set voxels of one row are one component on each
// side).  Intra-block seams use all 9 (dr, dx) (26-connectivity), block faces only (0, 0)
// (6-connectivity, block_faces.py:99-111).  Intra pairs go to the tile's slot list for k_block_uf
// (block-local ids), block-face pairs to the tile's inter list (node ids) for k_inter_union;
// edges and corners (intra only) go through stitch_tile.  Overflowing tiles are flagged: their
// block (big[]) or the tile itself (iovf[]) is handled by the global fallback k_stitch.
// ------------------------------------------------------------------------------------------
constexpr int TPI = 256;           // block-face pair slots per tile
constexpr int SEAM_HASH_BITS = 8, SEAM_HASH = 1 << SEAM_HASH_BITS;   // per-wave pair set

// bits 2k, 2k+1 of the result := bits sh, sh+1 of face entry k of an 8-entry LDS word
// (two 16-bit entries per u32, entry 2j in the low half)
__device__ __forceinline__ u32 pack8(uint4 v, int sh) {
    const u32 w[4] = {v.x, v.y, v.z, v.w};
    u32 r = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) r |= (((w[j] >> sh) & 3u) << (4 * j)) | (((w[j] >> (16 + sh)) & 3u) << (4 * j + 2));
    return r;
}

// The three lower seams at once, one voxel row per lane: lanes 0-31 the z seam (rows y, bits x),
// 32-47 the y seam (rows z, bits x), 48-63 the x seam (rows z, bits y).  mode[s]: 0 no seam,
// 1 inside the block (all 9 (dr, dx): 26-connectivity), 2 block face ((0, 0): 6-connectivity).
// Each lane packs its own row of both sides straight from the staged entries (voxel 2c + i of
// row r is bit FK_BITS + 2 (r & 1) + i of entry (r / 2, c)), 16-B LDS reads.
// EMIT(seam, kA, kB) once per run of contacts.
template <class EM>
__device__ __forceinline__ void seam_rows3(const face_t* S, const int mode[3], int lane, EM&& emit) {
    const int seam = lane < 32 ? 0 : lane < 48 ? 1 : 2;
    const int r = lane - (seam == 0 ? 0 : seam == 1 ? 32 : 48), nr = seam == 0 ? TY : TZ;
    const int stride = seam == 2 ? CY : CX;
    const face_t* FA = S + (seam == 0 ? F_ZLO : seam == 1 ? F_YLO : F_XLO);
    const face_t* FB = S + (seam == 0 ? F_ZHI : seam == 1 ? F_YHI : F_XHI);
    const int md = seam == 0 ? mode[0] : seam == 1 ? mode[1] : mode[2];
    static_assert(CX % 8 == 0 && CY % 8 == 0 && F_YLO % 8 == 0 && F_XLO % 8 == 0 && F_ZHI % 8 == 0 &&
                  F_YHI % 8 == 0 && F_XHI % 8 == 0, "16-B aligned face rows");
    u64 A = 0, B0 = 0;
    if (md) {
        const uint4* pa = reinterpret_cast<const uint4*>(FA + (r >> 1) * stride);
        const uint4* pb = reinterpret_cast<const uint4*>(FB + (r >> 1) * stride);
        const int sh = FK_BITS + 2 * (r & 1);
#pragma unroll
        for (int q = 0; q < CX / 8; ++q) {
            if (q < stride / 8) {
                A |= (u64)pack8(pa[q], sh) << (16 * q);
                B0 |= (u64)pack8(pb[q], sh) << (16 * q);
            }
        }
    }
    const int lm = lane > 0 ? lane - 1 : 0, lp = lane + 1 < 64 ? lane + 1 : 63;
    const u64 Bm_ = __shfl(B0, lm, 64), Bp_ = __shfl(B0, lp, 64);
    const u64 Am_ = __shfl(A, lm, 64), Ap_ = __shfl(A, lp, 64);
    const u64 Bm = r > 0 ? Bm_ : 0ull, Bp = r + 1 < nr ? Bp_ : 0ull;
    const u64 Am = r > 0 ? Am_ : 0ull, Ap = r + 1 < nr ? Ap_ : 0ull;
    if (!md || !A) return;
    const bool full26 = md == 1;
    // bit x := bit x + dx
    auto sh = [](u64 v, int dx) { return dx > 0 ? v >> 1 : dx < 0 ? v << 1 : v; };
    // the run starts of the nine contact directions j = (dr + 1) * 3 + dx + 1 first (unrolled,
    // constant shifts), then ONE emit site walking them as a rolled loop over the directions
    // that have a contact anywhere in the wave (nine inlined copies of the emit path made the
    // kernel 19 k instructions with 1.7 k SGPR spill / reload sites)
    u64 M[9];
    u32 nzj = 0;
#pragma unroll
    for (int dr = -1; dr <= 1; ++dr) {
        const u64 B = dr < 0 ? Bm : dr > 0 ? Bp : B0;
        const u64 Ad = dr < 0 ? Am : Ap;
#pragma unroll
        for (int dx = -1; dx <= 1; ++dx) {
            const int j = (dr + 1) * 3 + dx + 1;
            M[j] = 0;
            if ((dr || dx) && !full26) continue;
            // contact A_r[x] - B_{r+dr}[x+dx].  Voxels next to each other on one side of the seam
            // are one component of that tile, so the pair is also given by a contact of smaller
            // |dr| + |dx| when A_r[x+dx] or B_{r+dr}[x] is set (dx != 0: the (dr, 0) contact) or
            // A_{r+dr}[x] or B_r[x+dx] is set (dr != 0: the (0, dx) contact); by induction every
            // pair keeps a contact that is not dropped, and (0, 0) contacts never are.
            u64 C = A & sh(B, dx);
            if (dx) C &= ~(sh(A, dx) | B);
            if (dr) C &= ~(Ad | sh(B0, dx));
            u64 m0 = C & ~(C << 1);
            // a (0, 0) run starting where the row before also had a (0, 0) contact repeats that
            // contact's pair (rows r - 1 and r are adjacent on both sides): only the topmost emits
            if (!dr && !dx) m0 &= ~(Am & Bm);
            M[j] = m0;
            nzj |= m0 ? 1u << j : 0u;
        }
    }
    u32 la = NONE, lb = NONE;                                         // last pair emitted by this lane
#pragma unroll 1
    for (u32 todo = nzj; todo; todo &= todo - 1) {
        const int j = __builtin_ctz(todo);
        u64 m = 0;
#pragma unroll
        for (int i = 0; i < 9; ++i) m = i == j ? M[i] : m;
        const int dx = j % 3 - 1, rb = r + j / 3 - 1;
        for (; m; m &= m - 1) {
            const int x = __builtin_ctzll(m);
            const u32 ka = FA[(r >> 1) * stride + (x >> 1)] & FK_MASK;
            const u32 kb = FB[(rb >> 1) * stride + ((x + dx) >> 1)] & FK_MASK;
            if (ka == la && kb == lb) continue;             // cheap first filter
            la = ka; lb = kb;
            emit(seam, ka, kb);
        }
    }
}

// Face entries of the edge and corner neighbours inside the block (26-connectivity), staged in
// LDS with the face planes so that no dependent global load remains (0 where absent):
//   [0,32)   ZHI cube row (lyn-1)/2 of (-1,-1, 0)     [32,64)  ZHI cube row 0 of (-1,+1, 0)
//   [64,80)  ZHI cube column (lxn-1)/2 of (-1,0,-1)   [80,96)  ZHI cube column 0 of (-1,0,+1)
//   [96,104) YHI cube column (lxn-1)/2 of (0,-1,-1)   [104,112) YHI cube column 0 of (0,-1,+1)
//   [112,116) ZHI corner entries of (-1, s1, s2), index (s1 > 0) * 2 + (s2 > 0)
constexpr int EDGE_N = 128;

// Which of a tile's neighbours lie in its block (from the tile's block-local position; no table
// loads).  A lower neighbour inside the block is a full tile (only a block's last tile along an
// axis is truncated), so its facing row / column is row TY - 1 / column TX - 1.
struct InBlock {
    bool z, ym, yp, xm, xp;        // (-1, 0, 0), (0, -1, 0), (0, +1, 0), (0, 0, -1), (0, 0, +1)
    __device__ __forceinline__ bool y(int s) const { return s < 0 ? ym : yp; }
    __device__ __forceinline__ bool x(int s) const { return s < 0 ? xm : xp; }
};

__device__ __forceinline__ void stage_edges(const Geom& g, const face_t* __restrict__ FACES, int64_t t,
                                            const InBlock& nb, face_t* E, int lane) {
    const int64_t sz = (int64_t)g.nt[1] * g.nt[2], sy = g.nt[2];
    constexpr int YL = (TY - 1) / 2, XL = (TX - 1) / 2;          // facing cube row / column of a lower neighbour
#pragma unroll
    for (int i = lane; i < EDGE_N; i += 64) {
        u32 v = 0;
        if (i < 32) {
            if (nb.z && nb.ym) v = FACES[(t - sz - sy) * FACE_STRIDE + F_ZHI + YL * CX + i];
        } else if (i < 64) {
            if (nb.z && nb.yp) v = FACES[(t - sz + sy) * FACE_STRIDE + F_ZHI + (i - 32)];
        } else if (i < 80) {
            if (nb.z && nb.xm) v = FACES[(t - sz - 1) * FACE_STRIDE + F_ZHI + (i - 64) * CX + XL];
        } else if (i < 96) {
            if (nb.z && nb.xp) v = FACES[(t - sz + 1) * FACE_STRIDE + F_ZHI + (i - 80) * CX];
        } else if (i < 104) {
            if (nb.ym && nb.xm) v = FACES[(t - sy - 1) * FACE_STRIDE + F_YHI + (i - 96) * CX + XL];
        } else if (i < 112) {
            if (nb.ym && nb.xp) v = FACES[(t - sy + 1) * FACE_STRIDE + F_YHI + (i - 104) * CX];
        } else if (i < 116) {
            const int s1 = (i - 112) & 2 ? 1 : -1, s2 = (i - 112) & 1 ? 1 : -1;
            if (nb.z && nb.y(s1) && nb.x(s2))
                v = FACES[(t - sz + s1 * sy + s2) * FACE_STRIDE + F_ZHI + (s1 < 0 ? YL : 0) * CX + (s2 < 0 ? XL : 0)];
        }
        E[i] = (face_t)v;
    }
}

// Edge and corner seams as bit rows, one edge per lane (lanes 0-5), corners on lanes 6-9:
//   lane 0/1 (-1,-1,0)/(-1,+1,0): own ZLO row y = 0 / ly-1 against the neighbour's ZHI row, bits x
//   lane 2/3 (-1,0,-1)/(-1,0,+1): own ZLO column x = 0 / lx-1, bits y
//   lane 4/5 (0,-1,-1)/(0,-1,+1): own YLO column x = 0 / lx-1, bits z
// EMIT(oz, oy, ox, ka, kb) once per run of contacts (26-connectivity along the edge), the
// neighbour tile being t + oz sz + oy sy + ox.
template <class EM>
__device__ __forceinline__ void seam_edges_rows(const face_t* S, const face_t* E, const TileInfo& ti,
                                                const InBlock& nb, int lane, EM&& emit) {
    const int ncy = (ti.ly + 1) / 2, ncx = (ti.lx + 1) / 2;
    const bool zok = nb.z;
    auto yok = [&](int s) { return nb.y(s); };
    auto xok = [&](int s) { return nb.x(s); };
    auto ypar = [&](int s) { return s < 0 ? (TY - 1) & 1 : 0; };   // neighbour's facing y parity
    auto xpar = [&](int s) { return s < 0 ? (TX - 1) & 1 : 0; };
    const bool ok[6] = {zok && yok(-1), zok && yok(1), zok && xok(-1), zok && xok(1),
                        yok(-1) && xok(-1), yok(-1) && xok(1)};
    // own / neighbour rows of the six edges (ballots over the position p = lane), and I: the
    // voxels next to both ends of a contact in a lower face neighbour of this tile inside the
    // block (staged in S) -- own (z, y, x) [edge voxel p] and the neighbour's voxel are both
    // 26-adjacent to (z - 1, y, x) (z faces: t - sz's ZHI), (z, y - 1, x) (t - sy's YHI) or
    // (z, y, x - 1) (t - 1's XHI), at position p or p + d; the face seams of this tile and of that
    // neighbour connect the pair through it, so such an edge contact is dropped
    u64 A[6], B[6], I[6];
    {
        const int p = lane;
#pragma unroll
        for (int e = 0; e < 2; ++e) {                      // bits x
            const int s = e ? 1 : -1, cyo = s < 0 ? 0 : ncy - 1, jo = s < 0 ? 0 : (ti.ly - 1) & 1;
            const u32 ea = ok[e] ? S[F_ZLO + cyo * CX + (p >> 1)] : 0u, eb = ok[e] ? E[(e ? 32 : 0) + (p >> 1)] : 0u;
            A[e] = __ballot((ea >> (FK_BITS + jo * 2 + (p & 1))) & 1u);
            B[e] = __ballot((eb >> (FK_BITS + ypar(s) * 2 + (p & 1))) & 1u);
            const u32 iz = ok[e] ? S[F_ZHI + cyo * CX + (p >> 1)] : 0u;     // (z - 1, y_e, x)
            const u32 iy = (ok[e] && s < 0) ? S[F_YHI + (p >> 1)] : 0u;      // (z, y_e - 1, x), plane z = 0
            I[e] = __ballot(((iz >> (FK_BITS + jo * 2 + (p & 1))) | (iy >> (FK_BITS + (p & 1)))) & 1u);
        }
#pragma unroll
        for (int e = 2; e < 4; ++e) {                      // bits y
            const int s = e == 3 ? 1 : -1, cxo = s < 0 ? 0 : ncx - 1, io = s < 0 ? 0 : (ti.lx - 1) & 1;
            const bool in = ok[e] && p < TY;
            const u32 ea = in ? S[F_ZLO + (p >> 1) * CX + cxo] : 0u, eb = in ? E[(e == 3 ? 80 : 64) + (p >> 1)] : 0u;
            A[e] = __ballot((ea >> (FK_BITS + (p & 1) * 2 + io)) & 1u);
            B[e] = __ballot((eb >> (FK_BITS + (p & 1) * 2 + xpar(s))) & 1u);
            const u32 iz = in ? S[F_ZHI + (p >> 1) * CX + cxo] : 0u;          // (z - 1, y, x_e)
            const u32 ix = (in && s < 0) ? S[F_XHI + (p >> 1)] : 0u;          // (z, y, x_e - 1), plane z = 0
            I[e] = __ballot(((iz >> (FK_BITS + (p & 1) * 2 + io)) | (ix >> (FK_BITS + (p & 1)))) & 1u);
        }
#pragma unroll
        for (int e = 4; e < 6; ++e) {                      // bits z
            const int s = e == 5 ? 1 : -1, cxo = s < 0 ? 0 : ncx - 1, io = s < 0 ? 0 : (ti.lx - 1) & 1;
            const bool in = ok[e] && p < TZ;
            const u32 ea = in ? S[F_YLO + (p >> 1) * CX + cxo] : 0u, eb = in ? E[(e == 5 ? 104 : 96) + (p >> 1)] : 0u;
            A[e] = __ballot((ea >> (FK_BITS + (p & 1) * 2 + io)) & 1u);
            B[e] = __ballot((eb >> (FK_BITS + (p & 1) * 2 + xpar(s))) & 1u);
            const u32 iy = in ? S[F_YHI + (p >> 1) * CX + cxo] : 0u;          // (z, y - 1, x_e)
            const u32 ix = (in && s < 0) ? S[F_XHI + (p >> 1) * CY] : 0u;     // (z, y, x_e - 1), row y = 0
            I[e] = __ballot(((iy >> (FK_BITS + (p & 1) * 2 + io)) | (ix >> (FK_BITS + (p & 1) * 2))) & 1u);
        }
    }
    // one candidate row pair per lane: the edges on lanes 0-5, the corners on lanes 6-9 (a single
    // bit each side); contact p of own row -> own entry S[ab + (p >> 1) as], neighbour entry
    // E[bb + (q >> 1)]; one emit site (the loops stay rolled: a copy of the emit path per
    // direction would blow the kernel past the instruction cache)
    u64 a = 0, b = 0, im = 0;
    int ab = 0, as = 0, bb = 0, oz = 0, oy = 0, ox = 0;
    if (lane < 6) {
        const int e = lane;
#pragma unroll
        for (int i = 0; i < 6; ++i) if (i == e) { a = A[i]; b = B[i]; im = I[i]; }
        const int s = (e & 1) ? 1 : -1;
        // neighbour offset (oz, oy, ox): tn = t + oz sz + oy sy + ox
        oz = e < 4 ? -1 : 0; oy = e < 2 ? s : e < 4 ? 0 : -1; ox = e < 2 ? 0 : s;
        if (e < 2) { ab = F_ZLO + (s < 0 ? 0 : ncy - 1) * CX; as = 1; bb = e ? 32 : 0; }
        else if (e < 4) { ab = F_ZLO + (s < 0 ? 0 : ncx - 1); as = CX; bb = e == 3 ? 80 : 64; }
        else { ab = F_YLO + (s < 0 ? 0 : ncx - 1); as = CX; bb = e == 5 ? 104 : 96; }
    } else if (lane < 10 && zok) {                          // corners (-1, s1, s2)
        const int c = lane - 6, s1 = (c & 2) ? 1 : -1, s2 = (c & 1) ? 1 : -1;
        if (yok(s1) && xok(s2)) {
            const int cyo = s1 < 0 ? 0 : ncy - 1, cxo = s2 < 0 ? 0 : ncx - 1;
            const int jo = s1 < 0 ? 0 : (ti.ly - 1) & 1, io = s2 < 0 ? 0 : (ti.lx - 1) & 1;
            ab = F_ZLO + cyo * CX + cxo; bb = 112 + c;
            oz = -1; oy = s1; ox = s2;
            const bool hit = ((S[ab] >> FK_BITS) & fsel(jo, io)) && ((E[bb] >> FK_BITS) & fsel(ypar(s1), xpar(s2)));
            a = b = hit ? 1ull : 0ull;
        }
    }
    if (a && b) {
        u32 la = NONE, lb = NONE;
#pragma unroll 1
        for (int d = -1; d <= 1; ++d) {
            u64 C = a & (d > 0 ? b >> 1 : d < 0 ? b << 1 : b);
            // a diagonal contact a[p] - b[p + d] whose pair a (0) contact also gives (a[p + d] or
            // b[p] set: neighbours along the line are one component of their tile) is dropped
            if (d) C &= ~((d > 0 ? a >> 1 : a << 1) | b);
            C &= ~(im | (d > 0 ? im >> 1 : d < 0 ? im << 1 : im));    // through a face neighbour
            for (u64 m = C & ~(C << 1); m; m &= m - 1) {
                const int p = __builtin_ctzll(m), q = p + d;
                const u32 ka = S[ab + (p >> 1) * as] & FK_MASK, kb = E[bb + (q >> 1)] & FK_MASK;
                if (ka == la && kb == lb) continue;
                la = ka; lb = kb;
                emit(oz, oy, ox, ka, kb);
            }
        }
    }
}

// STOP (ablation harness only; 0 in the library): 1 staged, 2 + z seam, 3 + y seam, 4 + x seam
// Tiles [t_begin, t_end): the seams of a z-layer chunk only read faces of that chunk and the
// layers below it, so the library runs them on a side stream behind the k_spec chunks.
// list (nullable): the tiles are list[1 .. list[0]] instead of the range (seams redone after k_fix)
struct SeamsLDS {
    alignas(16) face_t S[SP_WAVES][FACE_STRIDE];
    u32 H[SP_WAVES][SEAM_HASH];
    face_t E[SP_WAVES][EDGE_N];
    u32 cnt[SP_WAVES][2];
};

// the seams of tile t (valid) for wave w; every wave of the workgroup calls it (one barrier)
template <int STOP = 0>
__device__ __forceinline__ void seams_tile(const Geom& g, const face_t* __restrict__ FACES, const u32* __restrict__ COUNT,
                                           u64* PAIRS, u32* PC, u8* big, u64* IPAIRS, u32* IPC, u8* iovf, int64_t t,
                                           bool valid, SeamsLDS& LS) {
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    auto& Sall = LS.S;
    auto& Hall = LS.H;
    auto& Eall = LS.E;
    auto& cnt = LS.cnt;
    face_t* S = Sall[w];
    u32* H = Hall[w];
    TileInfo ti;
    face_t* E = Eall[w];
    // block-local position of the own tile and the tile strides inside its block (a neighbour in
    // the same block at offset (oz, oy, ox) is lt_own + oz bny bnx + oy bnx + ox)
    int lz = 0, ly = 0, lx = 0, bny = 0, bnx_ = 0;
    InBlock nb{};
    // an empty tile (no foreground voxel: masked out or all background) touches nothing across
    // its seams -- every contact needs an own foreground voxel -- so it skips the whole walk
    const bool empty = valid && __builtin_amdgcn_readfirstlane(COUNT[t]) == 0;
    if (valid && !empty) {
        ti = tile_info(g, t);
        const int bz = g.tblk[0][ti.iz], by = g.tblk[1][ti.iy], bx = g.tblk[2][ti.ix];
        lz = ti.iz - g.bt0[0][bz]; ly = ti.iy - g.bt0[1][by]; lx = ti.ix - g.bt0[2][bx];
        bny = g.btn[1][by]; bnx_ = g.btn[2][bx];
        nb.z = lz > 0; nb.ym = ly > 0; nb.yp = ly + 1 < bny; nb.xm = lx > 0; nb.xp = lx + 1 < bnx_;
        stage_faces(g, FACES, t, ti, S, lane, 64);
        stage_edges(g, FACES, t, nb, E, lane);
    }
    for (int i = lane; i < SEAM_HASH; i += 64) H[i] = NONE;
    if (lane < 2) cnt[w][lane] = 0;
    __syncthreads();
    if (!valid) return;
    if (empty) {
        if (lane == 0) { PC[t] = 0; IPC[t] = 0; }
        return;
    }
    const u32 bnx = (u32)bnx_, bnyx = (u32)bny * bnx;
    const u32 lt_own = (u32)lz * bnyx + (u32)ly * bnx + (u32)lx;
    const u32 capu = (u32)g.cap;
    u64* out = PAIRS + t * TPC;
    u64* iout = IPAIRS + t * TPI;
    // wave-aggregated append of one pair per active lane to the intra (0) or inter (1) list
    // (used for the pairs beyond a lane's register stash only)
    auto append = [&](bool to_inter, u64 v) {
        const u64 act = __ballot(1), mi = __ballot(to_inter), ma = act & ~mi;
        u32 base_a = 0, base_i = 0;
        if (lane == (int)(__ffsll((unsigned long long)act) - 1)) {
            if (ma) base_a = atomicAdd(&cnt[w][0], (u32)__popcll(ma));
            if (mi) base_i = atomicAdd(&cnt[w][1], (u32)__popcll(mi));
        }
        base_a = __builtin_amdgcn_readfirstlane(base_a);
        base_i = __builtin_amdgcn_readfirstlane(base_i);
        const u64 below = (1ull << lane) - 1;
        if (to_inter) {
            const u32 pos = base_i + (u32)__popcll(mi & below);
            if (pos < TPI) iout[pos] = v;
        } else {
            const u32 pos = base_a + (u32)__popcll(ma & below);
            if (pos < TPC) out[pos] = v;
        }
    };
    // per-lane stash of the first STASH pairs in registers, written out by one set of ballots at
    // the end (the contact loops are divergent: a wave-wide append per contact costs a ballot /
    // atomic / readfirstlane round on the scalar unit every iteration)
    constexpr int STASH = 4;
    u64 st0 = 0, st1 = 0, st2 = 0, st3 = 0;
    int ns = 0;
    u32 kinds = 0;                                            // bit j: slot j goes to the inter list
    auto push = [&](bool to_inter, u64 v) {
        if (ns < STASH) {
            st0 = ns == 0 ? v : st0; st1 = ns == 1 ? v : st1;
            st2 = ns == 2 ? v : st2; st3 = ns == 3 ? v : st3;
            kinds |= (u32)to_inter << ns;
            ++ns;
        } else {
            append(to_inter, v);
        }
    };
    if (STOP == 1) return;
    // first sighting of (neighbour, ka, kb) in this tile? (LDS hash set; a full set lets
    // duplicates through, which the consumers tolerate).  code: the neighbour's direction,
    // dz * 9 + (dy + 1) * 3 + (dx + 1) for the neighbour t - dz sz + dy sy + dx (distinct
    // directions are distinct tiles)
    auto fresh = [&](u32 code, u32 ka, u32 kb) -> bool {
        const u32 key = (code << 24) | ((ka & 0xFFFu) << 12) | (kb & 0xFFFu);
        u32 h = (key * 0x9E3779B1u) >> (32 - SEAM_HASH_BITS);
        for (int probe = 0; probe < 32; ++probe) {
            const u32 old = atomicCAS(&H[h], NONE, key);
            if (old == NONE) return true;
            if (old == key) return false;
            h = (h + 1) & (SEAM_HASH - 1);
        }
        return true;
    };
    const int64_t sz = (int64_t)g.nt[1] * g.nt[2], sy = g.nt[2];
    // the three lower seams: neighbour tile, mode (0 none, 1 intra 26-conn, 2 block face 6-conn)
    const int mode[3] = {nb.z ? 1 : ti.iz > 0 ? 2 : 0, nb.ym ? 1 : ti.iy > 0 ? 2 : 0, nb.xm ? 1 : ti.ix > 0 ? 2 : 0};
    const int myseam = lane < 32 ? 0 : lane < 48 ? 1 : 2;
    const int64_t tn_l = t - (myseam == 0 ? sz : myseam == 1 ? sy : 1);
    const u32 code_l = myseam == 0 ? 13u : myseam == 1 ? 1u : 3u;    // (-1,0,0) / (0,-1,0) / (0,0,-1)
    const u32 ltn_l = lt_own - (myseam == 0 ? bnyx : myseam == 1 ? bnx : 1u);
    const int md_l = myseam == 0 ? mode[0] : myseam == 1 ? mode[1] : mode[2];
    seam_rows3(S, mode, lane, [&](int, u32 ka, u32 kb) {
        if (!fresh(code_l, ka, kb)) return;
        if (md_l == 1) push(false, ((u64)((lt_own << 12) | ka) << 32) | ((ltn_l << 12) | kb));
        else push(true, ((u64)((u32)t * capu + ka) << 32) | ((u32)tn_l * capu + kb));
    });
    if (STOP != 4) {
        // edges and corners inside the block
        seam_edges_rows(S, E, ti, nb, lane, [&](int oz, int oy, int ox, u32 k1, u32 k2) {
            const u32 code = (u32)(-oz * 9 + (oy + 1) * 3 + (ox + 1));
            if (!fresh(code, k1, k2)) return;
            const u32 lt_e = lt_own + (u32)(oz * (int)bnyx + oy * (int)bnx + ox);
            push(false, ((u64)((lt_own << 12) | k1) << 32) | ((lt_e << 12) | k2));
        });
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // the stashes: slot-major, lane order inside a slot, behind the overflow appends
    u32 na = __builtin_amdgcn_readfirstlane(cnt[w][0]), ni = __builtin_amdgcn_readfirstlane(cnt[w][1]);
    const u64 below = (1ull << lane) - 1;
#pragma unroll
    for (int j = 0; j < STASH; ++j) {
        const bool has = j < ns, inter = (kinds >> j) & 1u;
        const u64 mi = __ballot(has && inter), ma = __ballot(has && !inter);
        if (!(mi | ma)) break;
        const u64 v = j == 0 ? st0 : j == 1 ? st1 : j == 2 ? st2 : st3;
        if (has) {
            if (inter) {
                const u32 pos = ni + (u32)__popcll(mi & below);
                if (pos < TPI) iout[pos] = v;
            } else {
                const u32 pos = na + (u32)__popcll(ma & below);
                if (pos < TPC) out[pos] = v;
            }
        }
        na += (u32)__popcll(ma);
        ni += (u32)__popcll(mi);
    }
    if (lane == 0) {
        PC[t] = na < TPC ? na : TPC;
        if (na > TPC) { big[ti.block] = 1; big[g.n_blocks] = 1; }
        IPC[t] = ni < TPI ? ni : TPI;
        if (ni > TPI) { iovf[t] = 1; iovf[g.n_tiles] = 1; }
    }
}

template <int STOP = 0>
__global__ __launch_bounds__(SP_WAVES * 64) void k_seams(Geom g, const face_t* __restrict__ FACES,
                                                         const u32* __restrict__ COUNT, u64* PAIRS, u32* PC,
                                                         u8* big, u64* IPAIRS, u32* IPC, u8* iovf,
                                                         int64_t t_begin, int64_t t_end, const u32* list) {
    __shared__ SeamsLDS LS;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t idx = (int64_t)blockIdx.x * SP_WAVES + w;
    int64_t t = t_begin + idx;
    bool valid = t < t_end;
    if (list) {
        const u32 nl = __builtin_amdgcn_readfirstlane(list[0]);
        valid = idx < (int64_t)nl;
        t = valid ? (int64_t)__builtin_amdgcn_readfirstlane(list[1 + idx]) : 0;
    }
    seams_tile<STOP>(g, FACES, COUNT, PAIRS, PC, big, IPAIRS, IPC, iovf, t, valid, LS);
}

// the listed tiles list[1 .. list[0]] with a fixed grid (the count stays on the device: the
// one-read-back schedule); the loop's trip count is uniform per workgroup
__global__ __launch_bounds__(SP_WAVES * 64) void k_seams_list(Geom g, const face_t* __restrict__ FACES,
                                                              const u32* __restrict__ COUNT, u64* PAIRS,
                                                              u32* PC, u8* big, u64* IPAIRS, u32* IPC, u8* iovf,
                                                              const u32* list) {
    __shared__ SeamsLDS LS;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const u32 nl = __builtin_amdgcn_readfirstlane(list[0]);
#pragma nounroll
    for (int64_t i0 = (int64_t)blockIdx.x * SP_WAVES; i0 < (int64_t)nl; i0 += (int64_t)gridDim.x * SP_WAVES) {
        const int64_t idx = i0 + w;
        const bool valid = idx < (int64_t)nl;
        const int64_t t = valid ? (int64_t)__builtin_amdgcn_readfirstlane(list[1 + idx]) : 0;
        seams_tile<0>(g, FACES, COUNT, PAIRS, PC, big, IPAIRS, IPC, iovf, t, valid, LS);
        __syncthreads();
    }
}

// Emulation of the reference's "empty job" branch (merge_assignments.py:115-123 with
// block_faces.py:169-176, opt-in): bflag[b] = 1 iff block b has a 6-connected face pair with one
// of its upper neighbours, i.e. b contributes a pair to its block_faces job.  One wave per tile
// with a lower block face: own lower face entries against the neighbour's upper face entries
// (the same cube positions and bit layout on both sides).
__global__ __launch_bounds__(256) void k_block_face_flags(Geom g, const face_t* __restrict__ FACES, u8* bflag) {
    const int lane = threadIdx.x & 63;
    const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (t >= g.n_tiles) return;
    const TileInfo ti = tile_info(g, t);
    const int64_t sz = (int64_t)g.nt[1] * g.nt[2], sy = g.nt[2];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const int i = a == 0 ? ti.iz : a == 1 ? ti.iy : ti.ix;
        if (i == 0 || g.tblk[a][i] == g.tblk[a][i - 1]) continue;
        const int64_t tn = t - (a == 0 ? sz : a == 1 ? sy : 1);
        const int lo = a == 0 ? F_ZLO : a == 1 ? F_YLO : F_XLO, hi = a == 0 ? F_ZHI : a == 1 ? F_YHI : F_XHI;
        const int n = a == 0 ? F_Z : a == 1 ? F_Y : F_X;
        bool hit = false;
        for (int e = lane; e < n; e += 64)
            hit |= ((FACES[t * FACE_STRIDE + lo + e] >> FK_BITS) & (FACES[tn * FACE_STRIDE + hi + e] >> FK_BITS)) != 0;
        if (__ballot(hit) && lane == 0) bflag[tile_info(g, tn).block] = 1;
    }
}

// Block-face unions from the k_seams lists.  A wave takes 64 consecutive tiles and walks their
// lists as one flat sequence, one pair per lane (a wave per tile left most lanes idle and paid
// a dependent-load chain per tile); node pairs -> current roots (both finds together),
// duplicate root pairs dropped per wave, union keyed by rid (the smaller rid becomes the root).
// tpw tiles per wave (lanes >= tpw count no pairs): 64 for large volumes; 16 for small ones puts
// more waves on the dependent finds (C2 0.023 -> 0.016 ms; at C3 16 measured 0.060 vs 0.044 ms)
// iovf_any / scalars (nullable; the one-read-back schedule): an overflowed tile list raises
// RF_IOVF instead of a launch of the global-memory fallback (the run is redone synchronised)
__global__ __launch_bounds__(256) void k_inter_union(Geom g, const u64* __restrict__ IPAIRS,
                                                     const u32* __restrict__ IPC, u32* P,
                                                     const u64* __restrict__ K, int tpw, const u8* iovf_any,
                                                     u64* scalars) {
    const int lane = threadIdx.x & 63;
    if (iovf_any && blockIdx.x == 0 && threadIdx.x == 0 && *iovf_any) atomicOr(scalars + 3, RF_IOVF);
    const int64_t t0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * tpw;
    if (t0 >= g.n_tiles) return;
    const int64_t tl = t0 + lane;
    const u32 cnt = (lane < tpw && tl < g.n_tiles) ? IPC[tl] : 0u;
    u32 incl = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const u32 y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    const u32 total = __shfl(incl, 63, 64), excl = incl - cnt;
    for (u32 j = 0; j < total; j += 64) {
        const u32 q = j + lane;
        // owner tile of flat pair q: the last lane whose exclusive offset is <= q
        int lo = 0;
#pragma unroll
        for (int st = 32; st > 0; st >>= 1) {
            const u32 e = (u32)__shfl((int)excl, lo + st, 64);
            if (e <= q) lo += st;
        }
        const u32 eo = (u32)__shfl((int)excl, lo, 64);
        if (q < total) {
            const u64 pr = IPAIRS[(t0 + lo) * TPI + (q - eo)];
            u32 ra = (u32)(pr >> 32), rb = (u32)pr;
            gfind2(P, ra, rb);
            if (ra != rb && wave_first(((u64)ra << 32) | rb)) gunion_roots(P, K, ra, rb);
        }
    }
}

// Global-memory stitch, one wave per tile (keys: first voxel (intra) or rid (inter)).  INTER:
// tiles with a lower block-face seam; INTRA: only tiles of blocks the LDS path could not take
// (big[block] != 0).
template <bool INTER>
__global__ __launch_bounds__(SP_WAVES * 64) void k_stitch(Geom g, const face_t* __restrict__ FACES, u32* P,
                                                          const u64* __restrict__ K, const u8* __restrict__ big,
                                                          const u8* __restrict__ only) {
    __shared__ u32 Sall[SP_WAVES][FACE_STRIDE];
    // the common case is nothing to do: big[n_blocks] / only[n_tiles] are "any block / tile
    // flagged" (set with the per-block / per-tile flags), so a small grid reads one flag and
    // leaves; otherwise it walks every tile
    if (INTER ? (only && !only[g.n_tiles]) : !big[g.n_blocks]) return;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    u32* S = Sall[w];
    const u32 capu = (u32)g.cap;
    for (int64_t t0 = (int64_t)blockIdx.x * SP_WAVES; t0 < g.n_tiles; t0 += (int64_t)gridDim.x * SP_WAVES) {
        const int64_t t = t0 + w;
        bool active = t < g.n_tiles;
        TileInfo ti;
        if (active) {
            ti = tile_info(g, t);
            if (INTER)
                active = (!only || only[t]) && ((ti.iz > 0 && g.tblk[0][ti.iz] != g.tblk[0][ti.iz - 1]) ||
                         (ti.iy > 0 && g.tblk[1][ti.iy] != g.tblk[1][ti.iy - 1]) ||
                         (ti.ix > 0 && g.tblk[2][ti.ix] != g.tblk[2][ti.ix - 1]));
            else
                active = big[ti.block] != 0;
            if (active) stage_faces(g, FACES, t, ti, S, lane, 64);
        }
        __syncthreads();
        if (active)
            stitch_tile<INTER>(g, FACES, S, t, ti, lane, 64, [&](int64_t t1, u32 e1, int64_t t2, u32 e2) {
                const u32 a = (u32)(t1 * capu) + (e1 & FK_MASK), b = (u32)(t2 * capu) + (e2 & FK_MASK);
                if (wave_first(((u64)a << 32) | b)) gunion(P, K, a, b);
            });
        __syncthreads();
    }
}

__device__ __forceinline__ u32 lfind_k(lds_u32* par, u32 x) {
    volatile lds_u32* vp = par;
    u32 p = vp[x];
    while (p != x) {
        const u32 gp = vp[p];
        if (gp == p) return p;
        vp[x] = gp;
        x = gp;
        p = vp[x];
    }
    return x;
}

// link the root with the larger key under the root with the smaller key (keys unique)
__device__ __forceinline__ void lunion_key(lds_u32* par, const u64* key, u32 a, u32 b) {
    while (true) {
        a = lfind_k(par, a);
        b = lfind_k(par, b);
        if (a == b) return;
        if (key[a] < key[b]) { const u32 t = a; a = b; b = t; }
        if (__hip_atomic_compare_exchange_strong(&par[a], &a, b, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP))
            return;
    }
}

// largest lt in [0, n) with off[lt] <= i (off: exclusive scan in LDS, off[n] > i): the tile that
// holds flat element i (empty tiles share their offset with the next one and are skipped)
__device__ __forceinline__ int flat_tile(const u32* off, int n, u32 i) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (off[mid] <= i) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// The block's tiles are visited as flat index ranges (nodes, pairs) so that every global load of
// a phase is in flight at once; the per-tile loops this replaces waited on one tile at a time.
// RL / RCB (nullable): the block's roots in first-voxel order -- skimage's label order inside the
// block (block_components.py:179) -- as node ids in RL[b * SB_LCAP + rank], their count in RCB[b]
// (replaces the global count / collect / radix sort of every root when no block needed the
// global fallback)
__global__ __launch_bounds__(SB_THREADS) void k_block_uf(Geom g, const u32* __restrict__ COUNT,
                                                         const u64* __restrict__ PAIRS, const u32* __restrict__ PC,
                                                         u32* P, const u64* __restrict__ KEY, u8* big, u32* RL,
                                                         u32* RCB) {
    __shared__ u32 noff[SB_MAXT + 1];      // nodes of the block's tiles, exclusive scan
    __shared__ u32 poff[SB_MAXT + 1];      // intra pairs of the block's tiles, exclusive scan
    __shared__ u32 lpar[SB_LCAP];
    __shared__ u64 lkey[SB_LCAP];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t b = blockIdx.x;
    // a block left to the global fallback ranks no roots here (RCB is read by k_block_scan)
    if (big[b]) { if (tid == 0 && RCB) RCB[b] = 0; return; }
    const int bx = (int)(b % g.nb[2]), by = (int)((b / g.nb[2]) % g.nb[1]), bz = (int)(b / ((int64_t)g.nb[2] * g.nb[1]));
    const int iz0 = g.bt0[0][bz], iy0 = g.bt0[1][by], ix0 = g.bt0[2][bx];
    const int nz = g.btn[0][bz], ny = g.btn[1][by], nx = g.btn[2][bx];
    const int ntb = nz * ny * nx;
    if (ntb > SB_MAXT) {
        if (tid == 0) { big[b] = 1; big[g.n_blocks] = 1; if (RCB) RCB[b] = 0; }
        return;
    }
    auto tile_of = [&](int lt) -> int64_t {
        const int lx = lt % nx, ly = (lt / nx) % ny, lz = lt / (nx * ny);
        return ((int64_t)(iz0 + lz) * g.nt[1] + (iy0 + ly)) * g.nt[2] + (ix0 + lx);
    };
    for (int lt = tid; lt < ntb; lt += SB_THREADS) {
        const int64_t t = tile_of(lt);
        noff[lt] = COUNT[t];
        poff[lt] = PC[t];
    }
    __syncthreads();
    if (wave < 2) {                        // wave 0 scans the node counts, wave 1 the pair counts
        u32* arr = wave == 0 ? noff : poff;
        u32 run = 0;
        for (int c0 = 0; c0 < ntb; c0 += 64) {
            const int lt = c0 + lane;
            const u32 v = lt < ntb ? arr[lt] : 0;
            const u32 x = wave_incl_sum(v);
            if (lt < ntb) arr[lt] = run + x - v;
            run += (u32)__builtin_amdgcn_readlane((int)x, 63);
        }
        if (lane == 0) arr[ntb] = run;
    }
    __syncthreads();
    const u32 N = noff[ntb], M = poff[ntb];
    if (N > SB_LCAP) {
        if (tid == 0) { big[b] = 1; big[g.n_blocks] = 1; if (RCB) RCB[b] = 0; }
        return;
    }
    // the key and pair loads of UF_ILP iterations are issued together (the block's few workgroups
    // leave most CUs idle here: the phases are latency-bound, one global round trip per iteration)
    constexpr int UF_ILP = 4;
    for (u32 i0 = tid; i0 < N; i0 += UF_ILP * SB_THREADS) {
        u64 kv[UF_ILP];
#pragma unroll
        for (int j = 0; j < UF_ILP; ++j) {
            const u32 i = i0 + j * SB_THREADS;
            if (i < N) {
                const int lt = flat_tile(noff, ntb, i);
                kv[j] = KEY[(u64)tile_of(lt) * g.cap + (i - noff[lt])];
            }
        }
#pragma unroll
        for (int j = 0; j < UF_ILP; ++j) {
            const u32 i = i0 + j * SB_THREADS;
            if (i < N) { lpar[i] = i; lkey[i] = kv[j]; }
        }
    }
    __syncthreads();
    lds_u32* par = as_lds(lpar);
    for (u32 i0 = tid; i0 < M; i0 += UF_ILP * SB_THREADS) {
        u64 pv[UF_ILP];
#pragma unroll
        for (int j = 0; j < UF_ILP; ++j) {
            const u32 i = i0 + j * SB_THREADS;
            if (i < M) {
                const int lt = flat_tile(poff, ntb, i);
                pv[j] = PAIRS[tile_of(lt) * TPC + (i - poff[lt])];
            }
        }
#pragma unroll
        for (int j = 0; j < UF_ILP; ++j) {
            const u32 i = i0 + j * SB_THREADS;
            if (i < M) {
                const u32 a = (u32)(pv[j] >> 32), c = (u32)pv[j];
                lunion_key(par, lkey, noff[a >> 12] + (a & 0xFFFu), noff[c >> 12] + (c & 0xFFFu));
            }
        }
    }
    __syncthreads();
    for (u32 i = tid; i < N; i += SB_THREADS) {
        const u32 r = lfind_k(par, i);
        if (r != i) {
            const int lt = flat_tile(noff, ntb, i), lo = flat_tile(noff, ntb, r);
            P[(u64)tile_of(lt) * g.cap + (i - noff[lt])] = (u32)((u64)tile_of(lo) * g.cap + (r - noff[lo]));
        }
    }
    if (!RL) return;
    // roots sorted by first voxel: (key << 13 | local index) packed, compacted into lkey (the keys
    // of the roots are taken into registers first), bitonic sort in LDS
    static_assert(SB_LCAP <= (1 << 13) && KEY_BITS + 13 <= 64, "packed root keys");
    __shared__ u32 nroot;
    constexpr int PER = SB_LCAP / SB_THREADS;
    u64 mine[PER];
    if (tid == 0) nroot = 0;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const u32 i = tid + j * SB_THREADS;
        mine[j] = (i < N && lpar[i] == i) ? (lkey[i] << 13) | i : ~0ull;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PER; ++j)
        if (mine[j] != ~0ull) lkey[atomicAdd(&nroot, 1u)] = mine[j];
    __syncthreads();
    const u32 R = nroot;
    u32 R2 = 1;
    while (R2 < R) R2 <<= 1;
    for (u32 i = R + tid; i < R2; i += SB_THREADS) lkey[i] = ~0ull;
    __syncthreads();
    for (u32 k = 2; k <= R2; k <<= 1)
        for (u32 j = k >> 1; j > 0; j >>= 1) {
            for (u32 i = tid; i < R2; i += SB_THREADS) {
                const u32 l = i ^ j;
                if (l > i) {
                    const u64 a = lkey[i], c = lkey[l];
                    if ((a > c) == ((i & k) == 0)) { lkey[i] = c; lkey[l] = a; }
                }
            }
            __syncthreads();
        }
    for (u32 r = tid; r < R; r += SB_THREADS) {
        const u32 i = (u32)(lkey[r] & 0x1FFFu);
        const int lt = flat_tile(noff, ntb, i);
        RL[(u64)b * SB_LCAP + r] = (u32)((u64)tile_of(lt) * g.cap + (i - noff[lt]));
    }
    if (tid == 0) RCB[b] = R;
}

// Per-block root counts -> block values (n + 1, or 0 for an empty block: block_components.py:175-182),
// their exclusive scan (merge_offsets.py:115-120) and that of the root counts; scalars[0] = sum of
// the values, scalars[2] = number of roots, scalars[3] = whether any block took the global
// fallback (big[nb]) -- the host reads [2..3] in one copy.  One workgroup, chunks of SB_THREADS blocks.
// root_cap: capacity of the root arrays sized by the host before the count is known (the
// one-read-back schedule); more roots set bit 1 of scalars[3] (the run is redone host-synchronised)
__global__ __launch_bounds__(SB_THREADS) void k_block_scan(int64_t nb, const u32* __restrict__ RCB, u32* ROFFB,
                                                           u64* values, u64* offsets, const u8* big, u64* scalars,
                                                           u64 root_cap, u64* sum_out) {
    __shared__ u64 wsum[2][SB_THREADS / 64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    u64 carry_r = 0, carry_v = 0;
    for (int64_t b0 = 0; b0 < nb; b0 += SB_THREADS) {
        const int64_t b = b0 + tid;
        const u64 r = b < nb ? RCB[b] : 0ull, v = r ? r + 1 : 0ull;
        u64 xr = r, xv = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const u64 yr = __shfl_up(xr, o, 64), yv = __shfl_up(xv, o, 64);
            if (lane >= o) { xr += yr; xv += yv; }
        }
        if (lane == 63) { wsum[0][wave] = xr; wsum[1][wave] = xv; }
        __syncthreads();
        u64 br = 0, bv = 0, tr = 0, tv = 0;
#pragma unroll
        for (int w = 0; w < SB_THREADS / 64; ++w) {
            if (w < wave) { br += wsum[0][w]; bv += wsum[1][w]; }
            tr += wsum[0][w]; tv += wsum[1][w];
        }
        if (b < nb) {
            ROFFB[b] = (u32)(carry_r + br + xr - r);
            values[b] = v;
            offsets[b] = carry_v + bv + xv - v;
        }
        carry_r += tr; carry_v += tv;
        __syncthreads();
    }
    if (tid == 0) {
        scalars[0] = carry_v;
        scalars[2] = carry_r;
        scalars[3] = (big[nb] ? RF_BIG : 0ull) | (carry_r > root_cap ? RF_ROOTS : 0ull);
        if (sum_out) *sum_out = carry_v;                // the slab's sum for the allgather
    }
}

// k_block_scan and k_emit_roots in one launch for up to SCAN_EMIT_MAXB blocks (the one-read-back
// schedule): every workgroup b reads all the blocks' root counts (8 KB at most, from L2) and forms
// its own exclusive prefixes of the root counts and of the block values, then emits its roots as
// k_emit_roots; workgroup 0 writes the totals and flags as k_block_scan (one launch and its ~6 us
// of boundary fewer per volume / slab)
constexpr int64_t SCAN_EMIT_MAXB = 2048;
__global__ __launch_bounds__(256) void k_scan_emit(int64_t nb, const u32* __restrict__ RL, const u32* __restrict__ RCB,
                                                   u32* ROFFB, u64* values, u64* offsets, const u8* big, u64* scalars,
                                                   u64 root_cap, u64* sum_out, u64* KEY, u64* keys2, u32* vals2,
                                                   u32* seg_start, u32* seg_end) {
    __shared__ u64 red[4][4];
    const int64_t b = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    u64 s[4] = {0, 0, 0, 0};                 // prefix roots, prefix values, total roots, total values
    for (int64_t i = tid; i < nb; i += 256) {
        const u64 r = RCB[i], v = r ? r + 1 : 0ull;
        if (i < b) { s[0] += r; s[1] += v; }
        s[2] += r; s[3] += v;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) s[k] += __shfl_down(s[k], o, 64);
        if (lane == 0) red[k][wave] = s[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) s[k] = red[k][0] + red[k][1] + red[k][2] + red[k][3];
    const u32 R = RCB[b], off = (u32)s[0];
    if (tid == 0) {
        ROFFB[b] = off;
        values[b] = R ? (u64)R + 1 : 0ull;
        offsets[b] = s[1];
        seg_start[b] = off;
        seg_end[b] = off + R;
        if (b == 0) {
            scalars[0] = s[3];
            scalars[2] = s[2];
            scalars[3] = (big[nb] ? RF_BIG : 0ull) | (s[2] > root_cap ? RF_ROOTS : 0ull);
            if (sum_out) *sum_out = s[3];
        }
    }
    for (u32 r = tid; r < R && off + (u64)r < root_cap; r += 256) {
        const u32 node = RL[(u64)b * SB_LCAP + r];
        keys2[off + r] = ((u64)b << KEY_BITS) | KEY[node];
        vals2[off + r] = node;
        KEY[node] = s[1] + r + 1;                          // its reference id (k_assign_rid with base 0)
    }
}

// the sorted per-block root lists as the (key, node) arrays of the generic path: keys2 = block <<
// KEY_BITS | first voxel, vals2 = node, segment [seg_start, seg_end) of each block; offsets
// (nullable): each root's key becomes its reference id offsets[b] + rank + 1 (each root is read
// and written by its own thread only)
__global__ __launch_bounds__(256) void k_emit_roots(const u32* __restrict__ RL, const u32* __restrict__ RCB,
                                                    const u32* __restrict__ ROFFB, u64* KEY, const u64* offsets,
                                                    u64* keys2, u32* vals2, u32* seg_start, u32* seg_end,
                                                    u64 root_cap) {
    const int64_t b = blockIdx.x;
    const u32 R = RCB[b], off = ROFFB[b];
    for (u32 r = threadIdx.x; r < R && off + (u64)r < root_cap; r += 256) {
        const u32 node = RL[(u64)b * SB_LCAP + r];
        keys2[off + r] = ((u64)b << KEY_BITS) | KEY[node];
        vals2[off + r] = node;
        if (offsets) KEY[node] = offsets[b] + r + 1;      // its reference id (k_assign_rid with base 0)
    }
    if (threadIdx.x == 0) { seg_start[b] = off; seg_end[b] = off + R; }
}

constexpr int WAVES = NTHREADS / 64;

// block-local roots per tile (no atomics: counts, then an exclusive scan, then a collect that
// writes each tile's roots at its scanned offset in node order)
__global__ __launch_bounds__(NTHREADS) void k_count_roots(Geom g, const u32* COUNT, const u32* P, u32* RC) {
    const int64_t t = (int64_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
    if (t >= g.n_tiles) return;
    const u32 R = COUNT[t];
    const u32 base = (u32)(t * g.cap);
    u32 n = 0;
    for (u32 k = threadIdx.x & 63; k < R; k += 64) n += (P[base + k] == base + k);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o, 64);
    if ((threadIdx.x & 63) == 0) RC[t] = n;
}

__global__ __launch_bounds__(NTHREADS) void k_collect_roots(Geom g, const u32* COUNT, const u32* P, const u64* KEY,
                                                            const u32* ROFF, u64* keys, u32* vals) {
    const int64_t t = (int64_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
    if (t >= g.n_tiles) return;
    const u32 R = COUNT[t];
    if (R == 0) return;
    const int lane = threadIdx.x & 63;
    const TileInfo ti = tile_info(g, t);
    const u32 base = (u32)(t * g.cap);
    u32 pos = ROFF[t];
    for (u32 k0 = 0; k0 < R; k0 += 64) {
        const u32 k = k0 + lane;
        const bool is = k < R && P[base + k] == base + k;
        const u64 bal = __ballot(is);
        if (is) {
            const u32 p = pos + (u32)__popcll(bal & ((1ull << lane) - 1));
            keys[p] = ((u64)ti.block << KEY_BITS) | KEY[base + k];
            vals[p] = base + k;
        }
        pos += (u32)__popcll(bal);
    }
}

__global__ void k_segments(int64_t n, const u64* keys, u32* seg_start, u32* seg_end) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const u64 b = keys[i] >> KEY_BITS;
    if (i == 0 || (keys[i - 1] >> KEY_BITS) != b) seg_start[b] = (u32)i;
    if (i == n - 1 || (keys[i + 1] >> KEY_BITS) != b) seg_end[b] = (u32)(i + 1);
}

__global__ void k_values(int64_t nb, const u32* seg_start, const u32* seg_end, u64* values) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    const u64 n = seg_end[b] - seg_start[b];
    values[b] = n ? n + 1 : 0;                                // block_components.py:175-182
}

// scalars[0] = sum of block values (n_labels - 1 of this volume / slab), merge_offsets.py:120
__global__ void k_nlabels(int64_t nb, const u64* values, const u64* offsets, u64* scalars) {
    if (threadIdx.x == 0 && blockIdx.x == 0) scalars[0] = offsets[nb - 1] + values[nb - 1];
}

// z-slab sharding: this slab's ids start at `base` (sum of the values of the slabs before it)
__global__ void k_add_base(int64_t nb, u64* offsets, u64 base) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b < nb) offsets[b] += base;
}

__global__ void k_assign_rid(int64_t n, const u64* keys, const u32* vals, const u32* seg_start,
                             const u64* offsets, u64* KR) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const u64 b = keys[i] >> KEY_BITS;
    KR[vals[i]] = offsets[b] + (u64)(i - seg_start[b]) + 1;   // skimage label = rank + 1
}

// Seam mapping (multi-GPU): sorted distinct ids U[m] and their merged representative V[m].
__device__ __forceinline__ u64 apply_map(u64 v, const u64* U, const u64* V, int64_t m) {
    if (m == 0) return v;
    int64_t lo = 0, hi = m;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (U[mid] < v) lo = mid + 1; else hi = mid;
    }
    return (lo < m && U[lo] == v) ? V[lo] : v;
}

// Seam map of the one-read-back shard schedule: open addressing over the distinct seam ids
// (keys, EMPTY = ~0; capacity mask + 1, at most a quarter full), par = union-find over slots
// keyed by the ids (the smallest id of a set is its root), vals = the id of each slot's root.
constexpr u64 HM_EMPTY = ~0ull;
struct HashMap {
    u64* keys = nullptr;
    u32* par = nullptr;
    u32 mask = 0;
    __device__ __forceinline__ static u32 hash(u64 id) { return (u32)((id * 0x9E3779B97F4A7C15ull) >> 32); }
    // slot of id, inserted if absent (the table never fills: sized for every id of the pairs)
    __device__ __forceinline__ u32 insert(u64 id) const {
        u32 h = hash(id) & mask;
        while (true) {
            u64 cur = __hip_atomic_load(keys + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (cur == HM_EMPTY) {
                cur = atomicCAS((unsigned long long*)(keys + h), HM_EMPTY, (unsigned long long)id);
                if (cur == HM_EMPTY) return h;
            }
            if (cur == id) return h;
            h = (h + 1) & mask;
        }
    }
    // the representative of id (id itself when it is not on any seam): the key of its slot's root
    __device__ __forceinline__ u64 get(u64 id) const {
        u32 h = hash(id) & mask;
        while (true) {
            const u64 cur = keys[h];
            if (cur == id) return keys[gfind(par, h)];
            if (cur == HM_EMPTY) return id;
            h = (h + 1) & mask;
        }
    }
};

// the one read-back of a run (see phase_final), written by k_status after k_lut_all:
// out[0] = redo flags (the run's scalars[3]; with shards, OR over every slab's header plus
// RF_PAIRS when a slab had more pairs than cap and RF_CUBES when a slab's ids exceed the 28-bit
// cube form), [1] = largest pair count of a slab, [2] = sum over the slabs (or this volume) of
// the block values, [3] = this slab's id base, [4] = tiles k_fix relabelled, [5..8] =
// scalars[0..3], [16 ..) = values[nb], then offsets[nb] (+ base)
struct StatusArgs {
    u64* out = nullptr;          // nullptr: no status (the host-synchronised schedule)
    const u32* FIX = nullptr;
    const u64* all = nullptr;    // shards: every slab's pair buffer [world][cap + 1][2]
    int world = 0;
    u64 cap = 0;
    const u64* values = nullptr;
    const u64* offsets = nullptr;
    int64_t nb = 0;
};

__device__ __forceinline__ void write_status(const StatusArgs& sa, const u64* scalars, const u64* sums, u64 base) {
    const int tid = threadIdx.x;
    if (tid == 0) {
        u64 flags = scalars[3], mx = 0, tot = scalars[0];
        if (sa.all) {
            tot = 0;
            for (int w = 0; w < sa.world; ++w) {
                const u64* h = sa.all + (u64)w * 2 * (sa.cap + 1);
                flags |= h[1];
                mx = h[0] > mx ? h[0] : mx;
                tot += sums[w];
                if (sums[w] >= (1ull << 28) - 2) flags |= RF_CUBES;
            }
            if (mx > sa.cap) flags |= RF_PAIRS;
        }
        sa.out[0] = flags; sa.out[1] = mx; sa.out[2] = tot; sa.out[3] = base; sa.out[4] = sa.FIX[0];
        for (int k = 0; k < 4; ++k) sa.out[5 + k] = scalars[k];
    }
    for (int64_t i = tid; i < sa.nb; i += blockDim.x) {
        sa.out[16 + i] = sa.values[i];
        sa.out[16 + sa.nb + i] = sa.offsets[i] + base;
    }
}

// lut[i] = base + i for the ids of this volume (slab): i in [0, scalars[0]] (the last one is
// the slack id n_labels - 1 on the last slab, merge_offsets.py:120)
__global__ void k_lut_init(u64 cap, const u64* scalars, u64 base, u64* lut) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < cap && i <= scalars[0]) lut[i] = base + i;
}

// k_lut_init and k_lut in one launch: the LUT entry of every id of this volume (slab) -- a root's
// id maps to its component's representative, every other id (label 0 of a block, the slack id) to
// itself; lut holds cap >= scalars[0] + 1 entries.  sums (nullable; the one-read-back shard schedule): offsets and KR are
// this slab's own id space (base 0) and the global base = sum of sums[0 .. rank) is added here;
// hm (keys != nullptr): the seam map.
__global__ void k_lut_all(u64 cap, int64_t nb, u64 base, const u64* sums, int rank, const u64* __restrict__ offsets,
                          const u64* __restrict__ values, const u32* __restrict__ seg_start, const u32* __restrict__ vals,
                          u64 nvals, u32* P, const u64* KR, const u64* U, const u64* V, int64_t m, HashMap hm,
                          u64* lut, u64* scalars) {
    u64 gbase = base, obase = base;                           // ids = obase + i; reps + (gbase - obase)
    if (sums) {
        gbase = 0;
        for (int r = 0; r < rank; ++r) gbase += sums[r];
        obase = 0;
    }
    // workgroup = block (grid-stride over the blocks), thread = one of the block's ids: no search
    // for the block of an id.  Block b owns ids offsets[b] + [0, values[b]): + 0 its label 0, + r
    // its root of rank r - 1; the slack id scalars[0] (n_labels - 1) maps to itself.
    const u64 n = scalars[0] + 1 < cap ? scalars[0] + 1 : cap;
    u64 owned = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0 && n) lut[n - 1] = gbase + n - 1;
    for (int64_t b = blockIdx.x; b < nb; b += gridDim.x) {
        const u64 off = offsets[b] - obase, v = values[b];
        const u64 s0 = seg_start[b];
        for (u64 r = threadIdx.x; r < v; r += blockDim.x) {
            const u64 i = off + r;
            if (i >= n - 1) break;                            // capacity-bound (a run to be redone)
            u64 rep = gbase + i;
            const u64 vi = s0 + r - 1;                        // vals index (< nvals: the root arrays' size)
            if (r > 0 && vi < nvals) {
                const u32 node = vals[vi];
                const u32 root = gfind(P, node);
                const u64 kr = KR[root] + (gbase - obase);
                rep = hm.keys ? hm.get(kr) : apply_map(kr, U, V, m);
                owned += (root == node && rep == kr);         // components owned here
            }
            lut[i] = rep;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) owned += __shfl_xor(owned, o, 64);
    if ((threadIdx.x & 63) == 0 && owned) atomicAdd((unsigned long long*)&scalars[1], (unsigned long long)owned);
}

// the run's status (see StatusArgs) by one workgroup after k_lut_all (a last-workgroup count in
// k_lut_all needed an agent-scope fence per workgroup: an L2 write-back each on gfx950, +0.04 ms
// at C3's 256 blocks)
__global__ __launch_bounds__(256) void k_status(StatusArgs st, const u64* scalars, const u64* sums, int rank) {
    u64 gbase = 0;
    if (sums)
        for (int r = 0; r < rank; ++r) gbase += sums[r];
    write_status(st, scalars, sums, gbase);
}

__global__ void k_lut(int64_t n, const u32* vals, u32* P, const u64* KR, u64 base, const u64* U, const u64* V,
                      int64_t m, u64* lut, u64* scalars) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const u32 node = vals[i];
    const u32 r = gfind(P, node);
    const u64 rep = apply_map(KR[r], U, V, m);
    lut[KR[node] - base] = rep;
    if (r == node && rep == KR[r]) atomicAdd((unsigned long long*)&scalars[1], 1ull);   // components owned here
}

// final label of every node into FIN (a separate buffer).  LOCAL (stage-level block_components)
// writes the block-local skimage label rid - offset; the fused path does not run this kernel --
// k_pass2<true> resolves each tile component's label itself, reading KR without writing it.
template <bool LOCAL>
__global__ __launch_bounds__(NTHREADS) void k_finalize(Geom g, const u32* COUNT, u32* P, const u64* KR,
                                                       const u64* offsets, const u64* U, const u64* V,
                                                       int64_t m, u64* FIN) {
    const int64_t t = (int64_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
    if (t >= g.n_tiles) return;
    const u32 R = COUNT[t];
    if (R == 0) return;
    const u32 base = (u32)(t * g.cap);
    u64 off = 0;
    if (LOCAL) off = offsets[tile_info(g, t).block];
    for (u32 k = threadIdx.x & 63; k < R; k += 64) {
        const u32 node = base + k;
        const u64 v = KR[gfind(P, node)];
        FIN[node] = LOCAL ? v - off : apply_map(v, U, V, m);
    }
}

// ------------------------------------------------------------------------------------------
// z-slab seams (multi-GPU).  The bottom / top voxel plane of a slab as the current component
// id of each voxel (0 = background), from the ZLO / ZHI face planes of the first / last tile
// layer.  One workgroup per tile of that layer.
// ------------------------------------------------------------------------------------------
// OT = u64: the ids; OT = u32: id - sub + 1 (0 = background), the compact form sent over xGMI
template <bool TOP, class OT = u64>
__global__ __launch_bounds__(NTHREADS) void k_plane_labels(Geom g, const face_t* __restrict__ FACES, u32* P,
                                                           const u64* __restrict__ KR, OT* plane, u64 sub = 0) {
    const int64_t t = (TOP ? (int64_t)(g.nt[0] - 1) * g.nt[1] * g.nt[2] : 0) + blockIdx.x;
    const TileInfo ti = tile_info(g, t);
    const face_t* F = FACES + t * FACE_STRIDE + (TOP ? F_ZHI : F_ZLO);
    const u32 base = (u32)(t * g.cap);
    const int ncy = (ti.ly + 1) / 2, ncx = (ti.lx + 1) / 2;
    for (int e = threadIdx.x; e < ncy * CX; e += NTHREADS) {
        const int cy = e / CX, cx = e % CX;
        if (cx >= ncx) continue;
        const u32 a = F[e];
        u64 v = a ? KR[gfind(P, base + (a & FK_MASK))] : 0;
        if (sizeof(OT) == 4 && v) v = v - sub + 1;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int y = 2 * cy + j, x = 2 * cx + i;
                if (y < ti.ly && x < ti.lx)
                    plane[(int64_t)(ti.y0 + y) * g.X + ti.x0 + x] = ((a >> (FK_BITS + j * 2 + i)) & 1) ? (OT)v : (OT)0;
            }
    }
}

// pairs of ids facing each other across a seam (6-connectivity, block_faces.py:99-111).  A voxel
// whose pair equals that of the voxel before it (i - 1) or above it (i - X) is dropped: the first
// voxel of every distinct pair in index order always emits, so the sort + unique that follows
// sees every pair at least once but only ~ the pair regions' corners (the unfiltered plane gave
// millions of single-counter atomics, 3.2 ms for a 4096^2 seam).  Appends are wave-aggregated.
// k_seam_pairs: 256 threads, 8 consecutive plane voxels per thread per round, 4 rounds per
// workgroup (8192 voxels); appends collect in an LDS buffer and leave with one global atomic per
// workgroup -- the one-voxel-per-thread kernel took one atomic per 1024 voxels, serialised on the
// counter at ~24 ns each (0.10 ms of the 0.104 ms of a 2048^2 seam, profiles/r03_slabs8_c3.json)
constexpr int SEAM_PAIR_THREADS = 256, SPV = 8, SP_ROUNDS = 4, SP_BUF = 2 * SEAM_PAIR_THREADS * SPV;
constexpr int64_t SP_WG_VOXELS = (int64_t)SEAM_PAIR_THREADS * SPV * SP_ROUNDS;
// Readers of the upper plane for k_seam_pairs: raw(i) is compared between neighbours (0 =
// background), id(raw) is the global id.
struct UpperIds {                  // uint64 ids (single-process schedule, stage tests)
    const u64* p;
    __device__ __forceinline__ u64 raw(int64_t i, u32, u32) const { return p[i]; }
    __device__ __forceinline__ u64 id(u64 r) const { return r; }
    __device__ __forceinline__ int64_t width(int64_t X) const { return X; }
};
struct UpperIds32 {                // uint32 id - base + 1 per voxel
    const u32* p;
    u64 base;
    __device__ __forceinline__ u64 raw(int64_t i, u32, u32) const { return p[i]; }
    __device__ __forceinline__ u64 id(u64 r) const { return r - 1 + base; }
    __device__ __forceinline__ int64_t width(int64_t X) const { return X; }
};
struct UpperCubes32 {              // per 2x2 cube: (id - base + 1) << 4 | 4 voxel bits (y&1)*2 + (x&1)
    const u32* p;
    u64 base;
    u32 X, CXg;
    __device__ __forceinline__ u64 raw(int64_t, u32 y, u32 x) const {
        const u32 c = p[(y >> 1) * CXg + (x >> 1)];
        return ((c >> ((y & 1) * 2 + (x & 1))) & 1u) ? (u64)(c >> 4) : 0ull;
    }
    __device__ __forceinline__ u64 id(u64 r) const { return r - 1 + base; }
    __device__ __forceinline__ int64_t width(int64_t) const { return X; }     // (y, x) need the cube grid's X
};

// Facing voxel pairs of a seam (plane voxel i: upper id, lower id), both non-zero.  A pair equal to
// that of voxel i - 1 or i - X is not emitted (the first voxel of every distinct pair in index
// order always is).  counter[0] = pairs appended, counter[1] = the largest id emitted (it sizes the
// packed key of dedup_pairs).
// htab (optional): a device hash set of emitted pairs (key a << 32 | b, empty = ~0, hmask + 1 slots):
// a pair already in it is dropped, so only distinct pairs are appended -- a 2048^2 membrane seam
// emits ~47 k pairs after the i - 1 / i - X filters but holds ~150 distinct ones.  The slot is read
// before the CAS (the popular pairs' slots are read from L2 instead of serialising atomics on
// them).  Pairs with an id >= 2^32, or whose probe sequence is full, are appended anyway and
// counter[2] is flagged (the host then dedups by sorting).
constexpr int SEAM_HASH_PROBES = 64;
__device__ __forceinline__ int seam_hash_insert(u64* htab, u32 hmask, u64 key) {     // 1 new, 0 dup, -1 full
    u32 h = (u32)((key * 0x9E3779B97F4A7C15ull) >> 40) & hmask;
    for (int p = 0; p < SEAM_HASH_PROBES; ++p) {
        u64 cur = __builtin_nontemporal_load(htab + h);
        if (cur == key) return 0;
        if (cur == ~0ull) {
            cur = atomicCAS((unsigned long long*)(htab + h), ~0ull, (unsigned long long)key);
            if (cur == ~0ull) return 1;
            if (cur == key) return 0;
        }
        h = (h + 1) & hmask;
    }
    return -1;
}

template <class UP>
__global__ __launch_bounds__(SEAM_PAIR_THREADS) void k_seam_pairs(int64_t n, int64_t X, UP upper,
                                                                  const u64* __restrict__ lower, u64* pa, u64* pb,
                                                                  unsigned long long* counter, u64 cap, u64* htab,
                                                                  u32 hmask) {
    __shared__ u32 wcnt[SEAM_PAIR_THREADS / 64];
    __shared__ unsigned long long wmax[SEAM_PAIR_THREADS / 64];
    __shared__ unsigned long long gbase;
    __shared__ u64 bufa[SP_BUF], bufb[SP_BUF];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const bool vec = ((uintptr_t)lower & 15) == 0;
    X = upper.width(X);                                        // plane row width of the (y, x) walk
    const u32 Xu = (u32)X;
    u64 mx = 0;
    u32 nbuf = 0;
    auto flush = [&]() {
        if (threadIdx.x == 0) gbase = nbuf ? atomicAdd(counter, (unsigned long long)nbuf) : 0ull;
        __syncthreads();
        const unsigned long long b0 = gbase;
        for (u32 q = threadIdx.x; q < nbuf; q += SEAM_PAIR_THREADS)
            if (b0 + q < cap) { pa[b0 + q] = bufa[q]; pb[b0 + q] = bufb[q]; }
        __syncthreads();
        nbuf = 0;
    };
    for (int r = 0; r < SP_ROUNDS; ++r) {
        const int64_t i0 = (int64_t)blockIdx.x * SP_WG_VOXELS + ((int64_t)r * SEAM_PAIR_THREADS + threadIdx.x) * SPV;
        u64 lo[SPV], up[SPV];
        if (vec && i0 + SPV <= n) {
#pragma unroll
            for (int j = 0; j < SPV; j += 2) {
                const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(lower + i0 + j);
                lo[j] = v.x; lo[j + 1] = v.y;
            }
        } else {
#pragma unroll
            for (int j = 0; j < SPV; ++j) lo[j] = i0 + j < n ? lower[i0 + j] : 0ull;
        }
        // (y, x) of i0, then stepped (one 32-bit division per thread and round; planes < 2^32 voxels)
        u32 y = (u32)((u64)i0 / Xu), x = (u32)(i0 - (int64_t)y * X);
        u32 yy = y, xx = x;
#pragma unroll
        for (int j = 0; j < SPV; ++j) {
            up[j] = (i0 + j < n) ? upper.raw(i0 + j, yy, xx) : 0ull;
            if (++xx == Xu) { xx = 0; ++yy; }
        }
        // voxel i0 - 1: lane - 1's last one; the first lane of a wave loads it
        u64 pu = __shfl_up(up[SPV - 1], 1, 64), pl = __shfl_up(lo[SPV - 1], 1, 64);
        if (lane == 0) {
            pu = pl = 0;
            if (i0 > 0 && i0 - 1 < n) {
                const u32 py = x ? y : y - 1, px = x ? x - 1 : Xu - 1;
                pu = upper.raw(i0 - 1, py, px);
                pl = lower[i0 - 1];
            }
        }
        bool emit[SPV];
        u32 cnt = 0;
        yy = y; xx = x;
#pragma unroll
        for (int j = 0; j < SPV; ++j) {
            const int64_t i = i0 + j;
            const u64 u = up[j], b = lo[j];
            const u64 qu = j ? up[j - 1] : pu, ql = j ? lo[j - 1] : pl;
            bool e = i < n && u && b && !(qu == u && ql == b);
            if (e && i >= X && upper.raw(i - X, yy - 1, xx) == u && lower[i - X] == b) e = false;
            if (e && htab) {
                const u64 a = upper.id(u);
                if ((a | b) >> 32) {
                    atomicOr(counter + 2, 1ull);
                } else {
                    const int r = seam_hash_insert(htab, hmask, (a << 32) | b);
                    if (r < 0) atomicOr(counter + 2, 2ull);
                    e = r != 0;
                }
            }
            emit[j] = e;
            if (e) {
                const u64 a = upper.id(u);
                mx = a > mx ? a : mx;
                mx = b > mx ? b : mx;
                ++cnt;
            }
            if (++xx == Xu) { xx = 0; ++yy; }
        }
        u32 xs = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) { const u32 t = __shfl_up(xs, o, 64); if (lane >= o) xs += t; }
        if (lane == 63) wcnt[wave] = xs;
        __syncthreads();
        u32 wb = 0, tot = 0;
#pragma unroll
        for (int v = 0; v < SEAM_PAIR_THREADS / 64; ++v) { const u32 c = wcnt[v]; wb += v < wave ? c : 0u; tot += c; }
        __syncthreads();
        if (nbuf + tot > (u32)SP_BUF) flush();
        u32 pos = nbuf + wb + xs - cnt;
#pragma unroll
        for (int j = 0; j < SPV; ++j)
            if (emit[j]) { bufa[pos] = upper.id(up[j]); bufb[pos] = lo[j]; ++pos; }
        nbuf += tot;
    }
    __syncthreads();
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { const u64 t = __shfl_xor(mx, o, 64); mx = t > mx ? t : mx; }
    if (lane == 0) wmax[wave] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long gm = 0;
        for (int v = 0; v < SEAM_PAIR_THREADS / 64; ++v) gm = wmax[v] > gm ? wmax[v] : gm;
        if (gm) atomicMax(counter + 1, gm);
    }
    if (nbuf) flush();
}

// The top voxel plane as one u32 per 2x2 cube of the global cube grid (ceil(Y/2) x ceil(X/2);
// needs even tile origins, i.e. even block_shape[1:]): (id - sub + 1) << 4 | the cube's 4
// face-voxel bits, a quarter of the voxel plane's bytes.  One workgroup per top-layer tile.
// scalars (nullable): the one-read-back schedule (KR holds the slab's own ids, sub = 0) and its
// 28-bit check (scalars[0] = the slab's sum of block values; too many ids: RF_CUBES in scalars[3],
// plane unused)
__global__ __launch_bounds__(NTHREADS) void k_top_cubes(Geom g, const face_t* __restrict__ FACES, u32* P,
                                                        const u64* __restrict__ KR, u32* cubes, u64 sub,
                                                        u64* scalars) {
    if (scalars && scalars[0] >= (1ull << 28) - 2) {
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr((unsigned long long*)&scalars[3], (unsigned long long)RF_CUBES);
        return;
    }
    const int64_t t = (int64_t)(g.nt[0] - 1) * g.nt[1] * g.nt[2] + blockIdx.x;
    const TileInfo ti = tile_info(g, t);
    const face_t* F = FACES + t * FACE_STRIDE + F_ZHI;
    const u32 base = (u32)(t * g.cap);
    const int ncy = (ti.ly + 1) / 2, ncx = (ti.lx + 1) / 2;
    const int64_t CXg = (g.X + 1) / 2;
    for (int e = threadIdx.x; e < ncy * CX; e += NTHREADS) {
        const int cy = e / CX, cx = e % CX;
        if (cx >= ncx) continue;
        const u32 a = F[e];
        u32 w = 0;
        if (a) w = ((u32)(KR[gfind(P, base + (a & FK_MASK))] - sub + 1) << 4) | (a >> FK_BITS);
        cubes[(int64_t)(ti.y0 / 2 + cy) * CXg + ti.x0 / 2 + cx] = w;
    }
}

// ---- the one-read-back shard schedule (distributed.py fast path): everything below reads the
// allgathered per-slab sums and seam-pair headers from device memory ------------------------

// Seam pairs of this slab's bottom face against the slab below's top plane in the cube form
// (k_top_cubes), straight from the face planes of the bottom tile layer (no bottom voxel plane):
// a 2x2 face cube holds one component id on each side, so each cube gives at most one pair
// (upper id, lower id) when the two sides share a foreground voxel (6-connectivity,
// block_faces.py:99-111).  A pair equal to that of the cube before it in x or above it in y is
// dropped (the first cube of every distinct pair in raster order still emits), the rest go
// through the device hash set htab (key a << 32 | b; ids >= 2^32 or a full probe sequence are
// appended anyway: the replicated union-find takes duplicates), after a per-workgroup LDS set
// (the membrane component's pair recurs in every tile).  Ids: KR holds this slab's own ids
// (base 0); the global ones add the sums of the slabs below.  out = [cap + 1][2]: row 0 = (count,
// redo flags), written by k_seam_hdr from scalars[5] (the count; zeroed by the front clear in k_sample), then
// the pairs.  One workgroup per bottom-layer tile.
__global__ __launch_bounds__(NTHREADS) void k_seam_cube_pairs(Geom g, const face_t* __restrict__ FACES, u32* P,
                                                              const u64* __restrict__ KR, const u32* __restrict__ upper,
                                                              const u64* __restrict__ sums, int rank, u64* out, u64 cap,
                                                              u64* htab, u32 hmask, u64* scalars) {
    static_assert(CY * CX <= NTHREADS, "one face cube per thread");
    constexpr int LH = 1024;                         // per-workgroup pair set (LDS)
    __shared__ u64 pa[CY * CX], pb[CY * CX];
    __shared__ u64 lset[LH];
    const int64_t t = blockIdx.x;                    // bottom layer: tiles 0 .. nt[1] * nt[2] - 1
    const TileInfo ti = tile_info(g, t);
    const face_t* F = FACES + t * FACE_STRIDE + F_ZLO;
    const u32 base = (u32)(t * g.cap);
    u64 ubase = 0, own = 0;
    for (int r = 0; r < rank; ++r) {
        own += sums[r];
        if (r < rank - 1) ubase += sums[r];
    }
    const int ncy = (ti.ly + 1) / 2, ncx = (ti.lx + 1) / 2;
    const int64_t CXg = (g.X + 1) / 2;
    const int e = threadIdx.x, cy = e / CX, cx = e % CX;
    const int lane = e & 63;
    for (int i = e; i < LH; i += NTHREADS) lset[i] = ~0ull;
    // the pair of this thread's face cube: (upper id, lower id), both global; 0 = none
    u64 a = 0, b = 0;
    if (e < CY * CX && cy < ncy && cx < ncx) {
        const u32 f = F[e];
        const u32 c = f ? upper[(int64_t)(ti.y0 / 2 + cy) * CXg + ti.x0 / 2 + cx] : 0u;
        if (c & (f >> FK_BITS) & 0xFu) {
            a = (u64)(c >> 4) - 1 + ubase;
            b = KR[gfind(P, base + (f & FK_MASK))] + own;
        }
    }
    if (e < CY * CX) { pa[e] = a; pb[e] = b; }
    __syncthreads();
    // the cube before in x or above in y with the same pair: dropped (the first cube of every
    // distinct pair in raster order still emits); the rest through the workgroup's LDS set, then
    // the device set: only pairs new to both are appended
    bool emit = a && !(cx > 0 && pa[e - 1] == a && pb[e - 1] == b) && !(cy > 0 && pa[e - CX] == a && pb[e - CX] == b);
    if (emit && !((a | b) >> 32)) {
        const u64 key = (a << 32) | b;
        u32 h = (u32)((key * 0x9E3779B97F4A7C15ull) >> 40) & (LH - 1);
        for (int p = 0; p < 64; ++p) {
            const u64 old = atomicCAS((unsigned long long*)&lset[h], ~0ull, (unsigned long long)key);
            if (old == ~0ull) break;                 // new to the workgroup
            if (old == key) { emit = false; break; }
            h = (h + 1) & (LH - 1);
        }
        if (emit) emit = seam_hash_insert(htab, hmask, key) != 0;
    }
    const u64 bal = __ballot(emit);
    if (bal) {
        const int first = (int)(__ffsll((unsigned long long)bal) - 1);
        unsigned long long pos = 0;
        if (lane == first) pos = atomicAdd((unsigned long long*)&scalars[5], (unsigned long long)__popcll(bal));
        pos = __shfl(pos, first, 64) + (u64)__popcll(bal & ((1ull << lane) - 1));
        if (emit && pos < cap) { out[2 + 2 * pos] = a; out[3 + 2 * pos] = b; }
    }
}

// row 0 of a slab's pair buffer: (pairs appended by k_seam_cube_pairs -- 0 on slab 0, which has
// no slab below it --, the slab's redo flags)
__global__ void k_seam_hdr(const u64* scalars, u64* hdr) {
    if (threadIdx.x == 0 && blockIdx.x == 0) { hdr[0] = scalars[5]; hdr[1] = scalars[3]; }
}

// seam map over the allgathered pair buffers all[w] = [cap + 1][2] (w < world): clear, then
// insert both ids of every pair and union their slots (smallest id = root), then resolve
__global__ void k_map_clear(HashMap hm) {
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i <= hm.mask; i += (u64)gridDim.x * blockDim.x) {
        hm.keys[i] = HM_EMPTY;
        hm.par[i] = (u32)i;
    }
}

__global__ void k_map_build(HashMap hm, const u64* __restrict__ all, int world, u64 cap) {
    const u64 n = (u64)world * cap;
    for (u64 q = (u64)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (u64)gridDim.x * blockDim.x) {
        const u64 w = q / cap, j = q % cap;
        const u64* buf = all + w * 2 * (cap + 1);
        if (j >= buf[0]) continue;
        const u32 sa = hm.insert(buf[2 + 2 * j]), sb = hm.insert(buf[3 + 2 * j]);
        gunion(hm.par, hm.keys, sa, sb);
    }
}

// copy of the seam-pair ids with their largest value (atomicMax per workgroup into *mx): sizes the
// radix sort of phase_map (ids of a C3 run fit 12 bits: 2 passes instead of 8)
__global__ __launch_bounds__(256) void k_copy_max64(int64_t n, const u64* __restrict__ in, u64* out,
                                                    unsigned long long* mx) {
    __shared__ unsigned long long wm[4];
    u64 m = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const u64 v = in[i];
        out[i] = v;
        m = v > m ? v : m;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { const u64 t = __shfl_xor(m, o, 64); m = t > m ? t : m; }
    if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 4; ++w) m = wm[w] > m ? wm[w] : m;
        if (m) atomicMax(mx, (unsigned long long)m);
    }
}

// seam union-find over compact indices: pairs of ids -> indices into the sorted distinct ids
__global__ void k_pairs_to_index(int64_t n, const u64* pairs, const u64* U, int64_t m, u64* ip) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 2 * n) return;
    const u64 v = pairs[i];
    int64_t lo = 0, hi = m;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (U[mid] < v) lo = mid + 1; else hi = mid;
    }
    ip[i] = (u64)lo;
}

__global__ void k_map_values(int64_t m, const u64* U, const u64* root, u64* V) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) V[i] = U[root[i]];
}

// ------------------------------------------------------------------------------------------
// k_pass2: recompute the tile CCL from the bit rows and write the uint64 labels
// ------------------------------------------------------------------------------------------
constexpr int LABCAP = 2048;          // component labels cached in LDS

// store the two voxels (x, x+1) of one cube row segment; 16-B store when aligned
// (plain stores: non-temporal ones measured 0.3 ms slower over the 34 GB of C3)
// (HIP's ulonglong2 is only 8-B aligned, so this compiles to two dwordx2 stores per lane at 16-B
// stride; a 16-B aligned vector type giving one dwordx4 per lane measured slower: k_pass2 5.85 vs
// 5.50 ms at C3, same box)
__device__ __forceinline__ void store2(u64* __restrict__ out, int64_t idx, u64 v0, u64 v1, bool two, bool vec) {
    if (two && vec) {
#if CC_P2_NTSTORE
        typedef u64 v2u __attribute__((ext_vector_type(2)));
        __builtin_nontemporal_store(v2u{v0, v1}, reinterpret_cast<v2u*>(out + idx));
#else
        *reinterpret_cast<ulonglong2*>(out + idx) = make_ulonglong2(v0, v1);
#endif
    } else {
        out[idx] = v0;
        if (two) out[idx + 1] = v1;
    }
}

// UF (the fused path, in place of a k_finalize pass over all nodes): the final label of tile
// component k is apply_map(KR[root of its node]) (see below); the finds are issued before the tile CCL so
// their dependent loads overlap it.  !UF: FIN holds the label of every node (k_finalize<true>).
// With a seam map (m > 0, z-slab shards) the representative comes from the LUT k_lut_all built
// (lut[rid - base] = apply_map(rid) for every root id of this slab): one load instead of a binary
// search over the m mapped ids per component.
template <bool UF>
__global__ __launch_bounds__(NTHREADS) void k_pass2(Geom g, const u64* __restrict__ BITS, const u32* COUNT,
                                                    const u64* __restrict__ FIN, u32* P, const u64* lut, u64 id_base,
                                                    int64_t m, u64* __restrict__ out, int order,
                                                    const u64* id_base_dev, const u64* lut_last, u64 lut_n = ~0ull) {
    CC_KERNEL_PROBE
    __shared__ u64 rows[NROWS];             // split bit rows (see tile_ccl)
    __shared__ TileCCL T;
    __shared__ u64 lab[LABCAP];
    // tile order: 0 linear (x fastest), 1 z fastest (the host picks 1 for rows of >= 4096 voxels:
    // writing the 4096-wide C5 slabs in x-fastest order took 6.09-6.14 ms, z-fastest 5.36 ms;
    // C3's 2048-wide volume is the other way round, 5.60 vs 5.84 ms), 2 XCD-contiguous (rows of
    // labels not 128-B aligned, X % 16 != 0: see xcd_contig)
    // (3 y fastest, 4 / 5: z / y fastest over the XCD-contiguous order: A/B of the C5 slab's
    // 4096-wide rows, CC_PASS2_ORDER)
    int64_t t = blockIdx.x;
    if (order >= 4) t = xcd_contig(t, gridDim.x);
    if (order == 1 || order == 4) {
        const int64_t n0 = g.nt[0];
        t = (t % n0) * ((int64_t)g.nt[1] * g.nt[2]) + t / n0;
    } else if (order == 3 || order == 5) {
        const int64_t n1 = g.nt[1], n2 = g.nt[2], q = t / n1;
        t = (q / n2) * n1 * n2 + (t % n1) * n2 + q % n2;
    } else if (order == 2) {
        t = xcd_contig(t, gridDim.x);
    }
    const TileInfo ti = tile_info(g, t);
    const int tid = threadIdx.x;
    const u32 R = COUNT[t];
    const bool vec = ((ti.x0 | (int)(g.X & 1)) & 1) == 0;    // 16-B aligned pairs
    const int ncz = (ti.lz + 1) / 2, ncy = (ti.ly + 1) / 2, ncx = (ti.lx + 1) / 2;
    if (R == 0) {
        for (int c = tid; c < NC; c += NTHREADS) {
            const int cz = c / (CY * CX), cy = (c / CX) % CY, cx = c % CX;
            if (cz >= ncz || cy >= ncy || cx >= ncx) continue;
            const bool two = 2 * cx + 1 < ti.lx;
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                const int z = 2 * cz + (d >> 1), y = 2 * cy + (d & 1);
                if (z < ti.lz && y < ti.ly)
                    store2(out, ((int64_t)(ti.z0 + z) * g.Y + ti.y0 + y) * g.X + ti.x0 + 2 * cx, 0, 0, two, vec);
            }
        }
        return;
    }
    const u32 base = (u32)(t * g.cap);
    if (UF && id_base_dev) id_base = __builtin_amdgcn_readfirstlane(*id_base_dev);
    // lut_last (nullable): the LUT's last index on the device (the one-read-back shard schedule,
    // whose ids are only checked after the run: a run to be redone must not read past the LUT);
    // lut_n: the LUT's allocated entries -- on a run flagged RF_ROOTS the slab's sum of block values
    // exceeds them and roots past the root capacity keep their raw keys, so both bounds apply
    const u64 lmax = (UF && lut_last) ? min(*lut_last, lut_n - 1) : lut_n - 1;
    auto label = [&](u32 node) -> u64 {
        if (!UF) return FIN[node];
        const u64 v = FIN[gfind(P, node)];
        return m ? (v - id_base <= lmax ? lut[v - id_base] : v) : v;
    };
    constexpr int LPT = LABCAP / NTHREADS;
    u64 lv[LPT];
#pragma unroll
    for (int j = 0; j < LPT; ++j) {
        const u32 k = tid + j * NTHREADS;
        lv[j] = k < R ? label(base + k) : 0ull;
    }
    for (int i = tid; i < NROWS; i += NTHREADS) rows[i] = ld_once(BITS + t * NROWS + i);
    __syncthreads();
    tile_ccl(rows, T, (u32*)lab);
#pragma unroll
    for (int j = 0; j < LPT; ++j) {
        const u32 k = tid + j * NTHREADS;
        if (k < R) lab[k] = lv[j];
    }
    __syncthreads();
    for (int c = tid; c < NC; c += NTHREADS) {
        const int cz = c / (CY * CX), cy = (c / CX) % CY, cx = c % CX;
        if (cz >= ncz || cy >= ncy || cx >= ncx) continue;
        const int r = (2 * cz) * TY + 2 * cy;
        const u32 m = vpair(rows[r], cx) | (vpair(rows[r + 1], cx) << 2) | (vpair(rows[r + TY], cx) << 4) |
                      (vpair(rows[r + TY + 1], cx) << 6);
        u64 v = 0;
        if (m) {
            const u32 k = cube_k(T, c);
            if (k < LABCAP) v = lab[k];
            else v = UF ? label(base + k) : __builtin_nontemporal_load(FIN + base + k);
        }
        const bool two = 2 * cx + 1 < ti.lx;
#pragma unroll
        for (int d = 0; d < 4; ++d) {                 // (dz, dy) = (d >> 1, d & 1); bits 4dz + 2dy + dx
            const int z = 2 * cz + (d >> 1), y = 2 * cy + (d & 1);
            if (z < ti.lz && y < ti.ly) {
                const u32 b = m >> (2 * d);
                store2(out, ((int64_t)(ti.z0 + z) * g.Y + ti.y0 + y) * g.X + ti.x0 + 2 * cx,
                       (b & 1) ? v : 0, (b & 2) ? v : 0, two, vec);
            }
        }
    }
    CC_KERNEL_PROBE_END
}

// ------------------------------------------------------------------------------------------
// k_threshold: the reference Threshold task (thresholded_components/threshold.py:131-171):
// per-block normalize (volume_utils.py:98-105) and compare, written as uint8.  One workgroup
// per tile; the block parameters come from k_block_stats + k_block_params (the same exact
// foreground interval the labelling path uses).  float4 loads / uchar4 stores on full tiles.
// ------------------------------------------------------------------------------------------
// threshold of one tile with block parameters p (uint8 0 / 1)
__device__ __forceinline__ void threshold_tile(const Geom& g, const TileInfo& ti, const BlockParam& p,
                                               const float* __restrict__ in, float thr, int mode, u8* __restrict__ out) {
    const int tid = threadIdx.x;
    const int n = ti.lz * ti.ly;
    auto at = [&](int row, int x) { return ((int64_t)(ti.z0 + row / ti.ly) * g.Y + ti.y0 + row % ti.ly) * g.X + ti.x0 + x; };
    if (ti.lx == TX && ((g.X | ti.x0) & 3) == 0) {
        for (int i = tid; i < n * (TX / 4); i += NTHREADS) {
            const int64_t o = at(i / (TX / 4), 4 * (i % (TX / 4)));
            const float4 v = *reinterpret_cast<const float4*>(in + o);
            uchar4 r;
            r.x = voxel_pred(p, v.x, thr, mode); r.y = voxel_pred(p, v.y, thr, mode);
            r.z = voxel_pred(p, v.z, thr, mode); r.w = voxel_pred(p, v.w, thr, mode);
            *reinterpret_cast<uchar4*>(out + o) = r;
        }
    } else {
        for (int i = tid; i < n * ti.lx; i += NTHREADS) {
            const int64_t o = at(i / ti.lx, i % ti.lx);
            out[o] = voxel_pred(p, in[o], thr, mode);
        }
    }
}

__global__ __launch_bounds__(NTHREADS) void k_threshold(Geom g, const BlockParam* __restrict__ bp,
                                                        const float* __restrict__ in, float thr, int mode,
                                                        u8* __restrict__ out) {
    const int64_t t = blockIdx.x;
    const TileInfo ti = tile_info(g, t);
    threshold_tile(g, ti, uniform_bp(bp[ti.block]), in, thr, mode, out);
}

// Speculative Threshold task: ONE read of the input.  Like k_spec (the labelling front), every
// tile is thresholded with its block's guessed interval (k_sample + k_guess) while the exact block
// statistics and the tile's TB (nearest values around the guessed bounds) accumulate; then
// k_params_verify lists the tiles whose guessed bits are not exact and k_thr_fix rewrites only
// those from the input.  Blocks without a guess are read for statistics only here (their tiles
// are always listed).  SIDES as k_spec.
// one tile (any shape): the generic path of k_thr_spec
template <int SIDES>
__device__ __forceinline__ void thr_spec_tile(const Geom& g, const SpecArgs& sa, int64_t t, const float* __restrict__ in,
                                              u8* __restrict__ out, u32 (*red)[NTHREADS / 64]) {
    const TileInfo ti = tile_info(g, t);
    const BlockParam p = uniform_bp(sa.guess[ti.block]);
    if (p.kind != BP_INTERVAL) {
        stats_tile(g, ti, in, sa.smin, sa.smax, sa.sflag, red);
        __syncthreads();       // red is reused by the next tile of the workgroup
        return;
    }
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const u32 lo = p.lo, hi = p.hi;
    u32 mn = 0xFFFFFFFFu, mx = 0u, K1N = 0xFFFFFFFFu, K1X = 0u, K2N = 0xFFFFFFFFu, K2X = 0u;
    auto voxel = [&](float x) -> u8 {
        const u32 o = f2ord(__float_as_uint(x));
        mn = min(mn, o);
        mx = max(mx, o);
        if (SIDES & 1) { const u32 k = o - lo; K1N = min(K1N, k); K1X = max(K1X, k); }
        if (SIDES & 2) { const u32 k = hi - o; K2N = min(K2N, k); K2X = max(K2X, k); }
        return SIDES == 1 ? o >= lo : SIDES == 2 ? o <= hi : (o >= lo && o <= hi);
    };
    const int n = ti.lz * ti.ly;
    auto at = [&](int row, int x) { return ((int64_t)(ti.z0 + row / ti.ly) * g.Y + ti.y0 + row % ti.ly) * g.X + ti.x0 + x; };
    if (ti.lx == TX && ((g.X | ti.x0) & 3) == 0) {
        for (int i = tid; i < n * (TX / 4); i += NTHREADS) {
            const int64_t o = at(i / (TX / 4), 4 * (i % (TX / 4)));
            const float4 v = *reinterpret_cast<const float4*>(in + o);
            uchar4 r;
            r.x = voxel(v.x); r.y = voxel(v.y); r.z = voxel(v.z); r.w = voxel(v.w);
            *reinterpret_cast<uchar4*>(out + o) = r;
        }
    } else {
        for (int i = tid; i < n * ti.lx; i += NTHREADS) {
            const int64_t o = at(i / ti.lx, i % ti.lx);
            out[o] = voxel(in[o]);
        }
    }
    mn = wave_min(mn);
    mx = wave_max(mx);
    if (SIDES & 1) { K1N = wave_min(K1N); K1X = wave_max(K1X); }
    if (SIDES & 2) { K2N = wave_min(K2N); K2X = wave_max(K2X); }
    if (lane == 0) {
        red[0][wave] = mn; red[1][wave] = mx; red[2][wave] = K1N; red[3][wave] = K1X; red[4][wave] = K2N;
        red[5][wave] = K2X;
    }
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < NTHREADS / 64; ++w) {
            mn = min(mn, red[0][w]); mx = max(mx, red[1][w]);
            K1N = min(K1N, red[2][w]); K1X = max(K1X, red[3][w]); K2N = min(K2N, red[4][w]); K2X = max(K2X, red[5][w]);
        }
        atomicMin(sa.smin + ti.block, mn);
        atomicMax(sa.smax + ti.block, mx);
        if (mx > 0xFF800000u || mn < 0x007FFFFFu) atomicOr(sa.sflag + ti.block, 1u);    // NaN
        u32 A = 0u, B = 0xFFFFFFFFu, C = 0u, D = 0xFFFFFFFFu;      // as k_spec
        if (SIDES & 1) {
            if ((u64)K1N + lo < (1ull << 32)) B = K1N + lo;
            if ((u64)K1X + lo >= (1ull << 32)) A = K1X + lo;
        }
        if (SIDES & 2) {
            if (K2N <= hi) C = hi - K2N;
            if (K2X > hi) D = hi - K2X;
        }
        u32* tb = sa.TB + 4 * t;
        tb[0] = A; tb[1] = B; tb[2] = C; tb[3] = D;
    }
    __syncthreads();           // red is reused by the next tile of the workgroup
}

// TB of one tile from its reduced wrapped-distance statistics (as k_spec)
template <int SIDES>
__device__ __forceinline__ void thr_tile_tb(u32* tb, u32 lo, u32 hi, u32 K1N, u32 K1X, u32 K2N, u32 K2X) {
    u32 A = 0u, B = 0xFFFFFFFFu, C = 0u, D = 0xFFFFFFFFu;
    if (SIDES & 1) {
        if ((u64)K1N + lo < (1ull << 32)) B = K1N + lo;
        if ((u64)K1X + lo >= (1ull << 32)) A = K1X + lo;
    }
    if (SIDES & 2) {
        if (K2N <= hi) C = hi - K2N;
        if (K2X > hi) D = hi - K2X;
    }
    tb[0] = A; tb[1] = B; tb[2] = C; tb[3] = D;
}

// k_thr_spec: four x-adjacent tiles per workgroup.  The uint8 output rows of one tile are 64 B --
// half a 128-B line, the other half written by another workgroup at another time, which is what
// held the one-tile kernel at 2.5 TB/s of stores (profiles/r03_thr_spec.json).  When the four
// tiles are full, in one block and 16-B aligned, the workgroup treats them as one 16 x 32 x 256
// slab: a lane owns 16 consecutive voxels of a row (four float4 loads, ONE 16-B store), 16 lanes a
// 256-voxel row, a wave 4 rows of a plane, the 8 waves the 32 rows, 16 planes; statistics per lane,
// reduced per tile (a lane's voxels lie in tile (lane % 16) / 4).  Otherwise the tiles go one at a
// time through thr_spec_tile.
template <int SIDES>
__global__ __launch_bounds__(NTHREADS) void k_thr_spec(Geom g, SpecArgs sa, const float* __restrict__ in,
                                                       u8* __restrict__ out) {
    __shared__ u32 red[6][NTHREADS / 64];
    __shared__ u32 red4[6][4][NTHREADS / 64];
    const int64_t t0 = sa.t0 + 4 * (int64_t)blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    bool fast = t0 + 3 < g.n_tiles && (g.X & 15) == 0;
    TileInfo ti = tile_info(g, t0);
    if (fast) {
        const TileInfo tl = tile_info(g, t0 + 3);
        fast = (ti.ix & 3) == 0 && tl.iz == ti.iz && tl.iy == ti.iy && tl.block == ti.block && ti.lz == TZ &&
               ti.ly == TY && ti.lx == TX && tl.lx == TX && (ti.x0 & 15) == 0 &&
               sa.guess[ti.block].kind == BP_INTERVAL;
    }
    if (!fast) {
        for (int k = 0; k < 4 && t0 + k < g.n_tiles; ++k) thr_spec_tile<SIDES>(g, sa, t0 + k, in, out, red);
        return;
    }
    const BlockParam p = uniform_bp(sa.guess[ti.block]);
    const u32 lo = p.lo, hi = p.hi;
    u32 mn = 0xFFFFFFFFu, mx = 0u, K1N = 0xFFFFFFFFu, K1X = 0u, K2N = 0xFFFFFFFFu, K2X = 0u;
    auto fgp = [&](u32 o) -> u32 { return SIDES == 1 ? o >= lo : SIDES == 2 ? o <= hi : (o >= lo && o <= hi); };
    auto quad = [&](float4 v) -> u32 {
        const u32 o0 = f2ord(__float_as_uint(v.x)), o1 = f2ord(__float_as_uint(v.y));
        const u32 o2 = f2ord(__float_as_uint(v.z)), o3 = f2ord(__float_as_uint(v.w));
        mn = min(min(min(min(mn, o0), o1), o2), o3);
        mx = max(max(max(max(mx, o0), o1), o2), o3);
        if (SIDES & 1) {
            const u32 k0 = o0 - lo, k1 = o1 - lo, k2 = o2 - lo, k3 = o3 - lo;
            K1N = min(min(min(min(K1N, k0), k1), k2), k3);
            K1X = max(max(max(max(K1X, k0), k1), k2), k3);
        }
        if (SIDES & 2) {
            const u32 k0 = hi - o0, k1 = hi - o1, k2 = hi - o2, k3 = hi - o3;
            K2N = min(min(min(min(K2N, k0), k1), k2), k3);
            K2X = max(max(max(max(K2X, k0), k1), k2), k3);
        }
        return fgp(o0) | (fgp(o1) << 8) | (fgp(o2) << 16) | (fgp(o3) << 24);
    };
    const int64_t sz = g.Y * g.X;
    const int64_t o0 = ((int64_t)ti.z0 * g.Y + ti.y0 + 4 * wave + (lane >> 4)) * g.X + ti.x0 + 16 * (lane & 15);
    const float* pin = in + o0;
    u8* pout = out + o0;
#pragma unroll 2
    for (int z = 0; z < TZ; ++z) {
        const float4* q = reinterpret_cast<const float4*>(pin + z * sz);
        // (plain loads: non-temporal ones, as in k_spec, made this kernel 4.4 -> 5.7 ms,
        // profiles/r05_ab_ntload.txt)
        const float4 v0 = q[0], v1 = q[1], v2 = q[2], v3 = q[3];
        uint4 r;
        r.x = quad(v0); r.y = quad(v1); r.z = quad(v2); r.w = quad(v3);
        *reinterpret_cast<uint4*>(pout + z * sz) = r;
    }
    // reduce over the lanes of one tile: xor 1, 2 (the 4 lanes of a tile row), 16, 32 (the rows)
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        if (o == 4 || o == 8) continue;
        mn = min(mn, (u32)__shfl_xor(mn, o, 64));
        mx = max(mx, (u32)__shfl_xor(mx, o, 64));
        if (SIDES & 1) { K1N = min(K1N, (u32)__shfl_xor(K1N, o, 64)); K1X = max(K1X, (u32)__shfl_xor(K1X, o, 64)); }
        if (SIDES & 2) { K2N = min(K2N, (u32)__shfl_xor(K2N, o, 64)); K2X = max(K2X, (u32)__shfl_xor(K2X, o, 64)); }
    }
    if (lane < 16 && (lane & 3) == 0) {
        const int k = lane >> 2;
        red4[0][k][wave] = mn; red4[1][k][wave] = mx; red4[2][k][wave] = K1N; red4[3][k][wave] = K1X;
        red4[4][k][wave] = K2N; red4[5][k][wave] = K2X;
    }
    __syncthreads();
    if (tid < 4) {
        const int k = tid;
        mn = red4[0][k][0]; mx = red4[1][k][0]; K1N = red4[2][k][0]; K1X = red4[3][k][0]; K2N = red4[4][k][0];
        K2X = red4[5][k][0];
        for (int w = 1; w < NTHREADS / 64; ++w) {
            mn = min(mn, red4[0][k][w]); mx = max(mx, red4[1][k][w]);
            K1N = min(K1N, red4[2][k][w]); K1X = max(K1X, red4[3][k][w]);
            K2N = min(K2N, red4[4][k][w]); K2X = max(K2X, red4[5][k][w]);
        }
        atomicMin(sa.smin + ti.block, mn);
        atomicMax(sa.smax + ti.block, mx);
        if (mx > 0xFF800000u || mn < 0x007FFFFFu) atomicOr(sa.sflag + ti.block, 1u);    // NaN
        thr_tile_tb<SIDES>(sa.TB + 4 * (t0 + k), lo, hi, K1N, K1X, K2N, K2X);
    }
}

// the tiles k_params_verify listed (FIX[0] of them, ids in FIX[1..]) thresholded again with their
// block's exact parameters; a fixed grid walks the list (usually empty: the grid returns at once)
__global__ __launch_bounds__(NTHREADS) void k_thr_fix(Geom g, const u32* FIX, const BlockParam* __restrict__ bp,
                                                      const float* __restrict__ in, float thr, int mode,
                                                      u8* __restrict__ out) {
    const u32 n = __builtin_amdgcn_readfirstlane(FIX[0]);
    for (u32 i = blockIdx.x; i < n; i += gridDim.x) {
        const int64_t t = __builtin_amdgcn_readfirstlane(FIX[1 + i]);
        const TileInfo ti = uniform_ti(tile_info(g, t));
        threshold_tile(g, ti, uniform_bp(bp[ti.block]), in, thr, mode, out);
    }
}

// instantiate the templates used by the host side
#define CC_SPEC(M, S) \
    template __global__ void k_spec<M, S>(Geom, SpecArgs, const float*, const u8*, u64*, face_t*, u32*, u32*, u64*);
CC_SPEC(false, 1) CC_SPEC(false, 2) CC_SPEC(false, 3) CC_SPEC(true, 1) CC_SPEC(true, 2) CC_SPEC(true, 3)
#undef CC_SPEC
template __global__ void k_seams<0>(Geom, const face_t*, const u32*, u64*, u32*, u8*, u64*, u32*, u8*, int64_t, int64_t, const u32*);
template __global__ void k_stitch<false>(Geom, const face_t*, u32*, const u64*, const u8*, const u8*);
template __global__ void k_stitch<true>(Geom, const face_t*, u32*, const u64*, const u8*, const u8*);
template __global__ void k_finalize<true>(Geom, const u32*, u32*, const u64*, const u64*, const u64*, const u64*, int64_t, u64*);
template __global__ void k_plane_labels<false>(Geom, const face_t*, u32*, const u64*, u64*, u64);
template __global__ void k_plane_labels<true>(Geom, const face_t*, u32*, const u64*, u64*, u64);
template __global__ void k_plane_labels<true, u32>(Geom, const face_t*, u32*, const u64*, u32*, u64);

}  // namespace cc
