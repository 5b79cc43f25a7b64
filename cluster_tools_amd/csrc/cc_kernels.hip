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

// ------------------------------------------------------------------------------------------
// tile CCL in LDS.  rows[NROWS] holds the tile's foreground bits (zero outside its extent).
// After return (R = number of tile-local components): for every non-empty cube c,
//   root = par[c] & 0xFFFF, k = par[root] >> 16 (k in [0, R), deterministic).
// ------------------------------------------------------------------------------------------
__device__ u32 tile_ccl(const u64* rows, u8* cm, u32* par, u32* scratch) {
    const int tid = threadIdx.x;
    for (int c = tid; c < NC; c += NTHREADS) {
        const int cz = c / (CY * CX), cy = (c / CX) % CY, cx = c % CX;
        const int r = (2 * cz) * TY + 2 * cy;
        const int sh = 2 * cx;
        const u32 m = (u32)((rows[r] >> sh) & 3) | ((u32)((rows[r + 1] >> sh) & 3) << 2) |
                      ((u32)((rows[r + TY] >> sh) & 3) << 4) | ((u32)((rows[r + TY + 1] >> sh) & 3) << 6);
        cm[c] = (u8)m;
        par[c] = m ? (u32)c : NONE;
    }
    __syncthreads();
    for (int c = tid; c < NC; c += NTHREADS) {
        const u32 m = cm[c];
        if (!m) continue;
        const int cz = c / (CY * CX), cy = (c / CX) % CY, cx = c % CX;
#define CC_MERGE(DZ, DY, DX)                                                                   \
    {                                                                                          \
        const int nz = cz + (DZ), ny = cy + (DY), nx = cx + (DX);                              \
        if (nz >= 0 && ny >= 0 && ny < CY && nx >= 0 && nx < CX) {                            \
            const int n = c + (DZ) * (CY * CX) + (DY) * CX + (DX);                             \
            constexpr u32 SC = sel_bits(self_sel(DZ), self_sel(DY), self_sel(DX));             \
            constexpr u32 SN = sel_bits(nbr_sel(DZ), nbr_sel(DY), nbr_sel(DX));                \
            if ((m & SC) && (cm[n] & SN)) lunion(par, (u32)c, (u32)n);                          \
        }                                                                                      \
    }
        CC_DIRS(CC_MERGE)
#undef CC_MERGE
    }
    __syncthreads();
    for (int c = tid; c < NC; c += NTHREADS)
        if (cm[c]) par[c] = lfind(par, (u32)c);
    __syncthreads();
    u32 cnt = 0;
    for (int c = tid; c < NC; c += NTHREADS)
        cnt += (cm[c] && par[c] == (u32)c);
    u32 total;
    u32 k = block_excl_scan(cnt, scratch, &total);
    for (int c = tid; c < NC; c += NTHREADS)
        if (cm[c] && par[c] == (u32)c) par[c] = (u32)c | (k++ << 16);
    __syncthreads();
    return total;
}

__device__ __forceinline__ u32 cube_k(const u32* par, int c) {
    const u32 root = par[c] & 0xFFFFu;
    return par[root] >> 16;
}

// ------------------------------------------------------------------------------------------
// k_block_stats: per-block ordered min / max and NaN flag.  One workgroup per tile, lane = x.
// ------------------------------------------------------------------------------------------
constexpr int UNR = 16;   // rows in flight per wave

__global__ __launch_bounds__(NTHREADS) void k_block_stats(Geom g, const float* __restrict__ in,
                                                          u32* smin, u32* smax, u32* sflag) {
    __shared__ u32 red[3][NTHREADS / 64];
    const int64_t t = blockIdx.x;
    const TileInfo ti = tile_info(g, t);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nrows = ti.lz * ti.ly;
    u32 mn = 0xFFFFFFFFu, mx = 0u;
    bool nan = false;
    const bool act = lane < ti.lx;
    for (int r0 = wave * UNR; r0 < nrows; r0 += (NTHREADS / 64) * UNR) {
        float v[UNR];
#pragma unroll
        for (int j = 0; j < UNR; ++j) {
            const int r = r0 + j;
            v[j] = 0.0f;
            if (act && r < nrows) {
                const int z = ti.z0 + r / ti.ly, y = ti.y0 + r % ti.ly;
                v[j] = in[((int64_t)z * g.Y + y) * g.X + ti.x0 + lane];
            }
        }
#pragma unroll
        for (int j = 0; j < UNR; ++j) {
            if (act && r0 + j < nrows) {
                const float x = v[j];
                if (x != x) nan = true;
                else {
                    const u32 o = f2ord(__float_as_uint(x));
                    mn = o < mn ? o : mn;
                    mx = o > mx ? o : mx;
                }
            }
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const u32 a = __shfl_xor(mn, o, 64), b = __shfl_xor(mx, o, 64);
        mn = a < mn ? a : mn;
        mx = b > mx ? b : mx;
    }
    const bool anynan = __any(nan);
    if (lane == 0) { red[0][wave] = mn; red[1][wave] = mx; red[2][wave] = anynan; }
    __syncthreads();
    if (threadIdx.x == 0) {
        u32 a = red[0][0], b = red[1][0], f = red[2][0];
        for (int w = 1; w < NTHREADS / 64; ++w) {
            a = red[0][w] < a ? red[0][w] : a;
            b = red[1][w] > b ? red[1][w] : b;
            f |= red[2][w];
        }
        atomicMin(smin + ti.block, a);
        atomicMax(smax + ti.block, b);
        if (f) atomicOr(sflag + ti.block, 1u);
    }
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

__global__ void k_block_params(int64_t nb, const u32* smin, const u32* smax, const u32* sflag,
                               float thr, int mode, BlockParam* bp) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    BlockParam p;
    p.kind = BP_EMPTY; p.lo = 1; p.hi = 0; p.pad = 0;
    const u32 omn = smin[b], omx = smax[b];
    const float mn = __uint_as_float(ord2f(omn)), mx = __uint_as_float(ord2f(omx));
    p.mn = mn;
    p.m = 0.0f;
    if (sflag[b] & 1u) { bp[b] = p; return; }                 // NaN anywhere: numpy min is NaN
    if (isinf(mn) || isinf(mx)) {
        p.kind = BP_EXACT;
        p.m = isinf(mn) ? __uint_as_float(0x7FC00000u) : mx - mn;
        bp[b] = p;
        return;
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
    bp[b] = p;
}

// ------------------------------------------------------------------------------------------
// shared: load the tile's foreground bit rows (threshold + mask) into LDS
// ------------------------------------------------------------------------------------------
template <bool HAS_MASK>
__device__ __forceinline__ void load_rows(const Geom& g, const TileInfo& ti, const float* __restrict__ in,
                                          const u8* __restrict__ mask, const BlockParam& p, float thr,
                                          int mode, u64* rows) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nrows = ti.lz * ti.ly;
    const bool act = lane < ti.lx;
    for (int r0 = wave * UNR; r0 < nrows; r0 += (NTHREADS / 64) * UNR) {
        float v[UNR];
        u8 mk[UNR];
#pragma unroll
        for (int j = 0; j < UNR; ++j) {
            const int r = r0 + j;
            v[j] = 0.0f;
            mk[j] = 0;
            if (act && r < nrows) {
                const int z = ti.z0 + r / ti.ly, y = ti.y0 + r % ti.ly;
                const int64_t idx = ((int64_t)z * g.Y + y) * g.X + ti.x0 + lane;
                v[j] = in[idx];
                if (HAS_MASK) mk[j] = mask[idx];
            }
        }
#pragma unroll
        for (int j = 0; j < UNR; ++j) {
            const int r = r0 + j;
            bool fg = act && r < nrows && voxel_pred(p, v[j], thr, mode);
            if (HAS_MASK) fg = fg && mk[j] != 0;
            const u64 bal = __ballot(fg);
            if (lane == 0 && r < nrows) rows[(r / ti.ly) * TY + (r % ti.ly)] = bal;
        }
    }
}

// face plane entry i of a tile (see cc_common.hpp for the layout)
__device__ __forceinline__ u32 face_entry(int i, const u64* rows, const u32* par, const TileInfo& ti) {
    u32 bits = 0;
    int c = 0;
    if (i < F_YLO) {                       // z faces: (cy, cx), bits (y-local j)*2 + (x-local i)
        const bool hi = i >= F_ZHI;
        const int e = hi ? i - F_ZHI : i;
        const int cy = e / CX, cx = e % CX;
        if (2 * cy >= ti.ly || 2 * cx >= ti.lx) return 0;
        const int z = hi ? ti.lz - 1 : 0;
        const u64 r0 = rows[z * TY + 2 * cy], r1 = rows[z * TY + 2 * cy + 1];
        bits = (u32)((r0 >> (2 * cx)) & 3) | ((u32)((r1 >> (2 * cx)) & 3) << 2);
        c = ((z >> 1) * CY + cy) * CX + cx;
    } else if (i < F_XLO) {                // y faces: (cz, cx), bits (z-local)*2 + (x-local)
        const bool hi = i >= F_YHI;
        const int e = hi ? i - F_YHI : i - F_YLO;
        const int cz = e / CX, cx = e % CX;
        if (2 * cz >= ti.lz || 2 * cx >= ti.lx) return 0;
        const int y = hi ? ti.ly - 1 : 0;
        const u64 r0 = rows[(2 * cz) * TY + y], r1 = rows[(2 * cz + 1) * TY + y];
        bits = (u32)((r0 >> (2 * cx)) & 3) | ((u32)((r1 >> (2 * cx)) & 3) << 2);
        c = (cz * CY + (y >> 1)) * CX + cx;
    } else {                               // x faces: (cz, cy), bits (z-local)*2 + (y-local)
        const bool hi = i >= F_XHI;
        const int e = hi ? i - F_XHI : i - F_XLO;
        const int cz = e / CY, cy = e % CY;
        if (2 * cz >= ti.lz || 2 * cy >= ti.ly) return 0;
        const int x = hi ? ti.lx - 1 : 0;
        const int r = (2 * cz) * TY + 2 * cy;
        bits = (u32)((rows[r] >> x) & 1) | ((u32)((rows[r + 1] >> x) & 1) << 1) |
               ((u32)((rows[r + TY] >> x) & 1) << 2) | ((u32)((rows[r + TY + 1] >> x) & 1) << 3);
        c = (cz * CY + cy) * CX + (x >> 1);
    }
    if (!bits) return 0;
    return cube_k(par, c) | (bits << 16);
}

// ------------------------------------------------------------------------------------------
// k_pass1: bit rows, tile-local components, their first voxels, face planes
// ------------------------------------------------------------------------------------------
template <bool HAS_MASK>
__global__ __launch_bounds__(NTHREADS) void k_pass1(Geom g, const float* __restrict__ in,
                                                    const u8* __restrict__ mask, const BlockParam* bp,
                                                    float thr, int mode, u64* BITS, u32* FACES,
                                                    u32* COUNT, u32* P, u64* KEY) {
    __shared__ u64 rows[NROWS];
    __shared__ u8 cm[NC];
    __shared__ u32 par[NC];
    __shared__ u32 key[NC];
    __shared__ u32 scratch[8];
    const int64_t t = blockIdx.x;
    const TileInfo ti = tile_info(g, t);
    const BlockParam p = bp[ti.block];
    const int tid = threadIdx.x;
    for (int i = tid; i < NROWS; i += NTHREADS) rows[i] = 0;
    __syncthreads();
    if (p.kind != BP_EMPTY) load_rows<HAS_MASK>(g, ti, in, mask, p, thr, mode, rows);
    __syncthreads();
    for (int i = tid; i < NROWS; i += NTHREADS) BITS[t * NROWS + i] = rows[i];
    const u32 R = tile_ccl(rows, cm, par, scratch);
    for (u32 k = tid; k < R; k += NTHREADS) key[k] = NONE;
    __syncthreads();
    for (int c = tid; c < NC; c += NTHREADS) {
        const u32 m = cm[c];
        if (!m) continue;
        const int cz = c / (CY * CX), cy = (c / CX) % CY, cx = c % CX;
        const int bi = __builtin_ctz(m);
        const int lz = 2 * cz + (bi >> 2), ly = 2 * cy + ((bi >> 1) & 1), lx = 2 * cx + (bi & 1);
        atomicMin(&key[cube_k(par, c)], (u32)((lz * TY + ly) * TX + lx));
    }
    __syncthreads();
    if (tid == 0) COUNT[t] = R;
    const u32 base = (u32)(t * g.cap);
    for (u32 k = tid; k < R; k += NTHREADS) {
        const u32 node = base + k;
        const u32 idx = key[k];
        const int lz = idx / (TY * TX), ly = (idx / TX) % TY, lx = idx % TX;
        P[node] = node;
        KEY[node] = ((u64)(g.zoff + ti.z0 + lz) * (u64)g.Y + (u64)(ti.y0 + ly)) * (u64)g.X + (u64)(ti.x0 + lx);
    }
    u32* F = FACES + t * FACE_STRIDE;
    for (int i = tid; i < FACE_STRIDE; i += NTHREADS) F[i] = face_entry(i, rows, par, ti);
}

// ------------------------------------------------------------------------------------------
// k_stitch<INTER>: unions across tile seams.
//   INTER = false: seams inside one block, 26-connectivity (13 tile directions).
//   INTER = true : seams on block faces, 6-connectivity (3 face directions).
// Keys: first-voxel index (intra) or rid (inter); the union keeps the smaller key as root.
// ------------------------------------------------------------------------------------------
template <bool INTER>
__global__ __launch_bounds__(NTHREADS) void k_stitch(Geom g, const u32* __restrict__ FACES, u32* P,
                                                     const u64* __restrict__ K) {
    const int64_t t = blockIdx.x;
    const TileInfo ti = tile_info(g, t);
    const int tid = threadIdx.x;
    const int64_t sz = (int64_t)g.nt[1] * g.nt[2], sy = g.nt[2];
    const u32 capu = (u32)g.cap;
    const u32* F = FACES + t * FACE_STRIDE;
    const int ncy = (ti.ly + 1) / 2, ncx = (ti.lx + 1) / 2, ncz = (ti.lz + 1) / 2;
    const u32 base = (u32)(t * g.cap);
    auto node_of = [&](int64_t tt, u32 e) -> u32 { return (u32)(tt * capu) + (e & 0xFFFFu); };

    // ---------------- z-lower seam ----------------
    if (ti.iz > 0) {
        const bool same_z = g.tblk[0][ti.iz] == g.tblk[0][ti.iz - 1];
        const int64_t tn = t - sz;
        const u32* FN = FACES + tn * FACE_STRIDE;
        if (INTER) {
            if (!same_z)
                for (int e = tid; e < ncy * CX; e += NTHREADS) {
                    const int cy = e / CX, cx = e % CX;
                    if (cx >= ncx) continue;
                    const u32 a = F[F_ZLO + e];
                    if (!a) continue;
                    const u32 b = FN[F_ZHI + e];
                    if ((a >> 16) & (b >> 16)) gunion(P, K, base + (a & 0xFFFFu), node_of(tn, b));
                    (void)cy;
                }
        } else if (same_z) {
            // face (-1, 0, 0): 9 cube offsets in (dy, dx)
            for (int e = tid; e < ncy * CX; e += NTHREADS) {
                const int cy = e / CX, cx = e % CX;
                if (cx >= ncx) continue;
                const u32 a = F[F_ZLO + e];
                if (!a) continue;
                const u32 ab = a >> 16;
                for (int dy = -1; dy <= 1; ++dy) {
                    const int ny = cy + dy;
                    if (ny < 0 || ny >= ncy) continue;
                    for (int dx = -1; dx <= 1; ++dx) {
                        const int nx = cx + dx;
                        if (nx < 0 || nx >= ncx) continue;
                        const u32 b = FN[F_ZHI + ny * CX + nx];
                        if (!b) continue;
                        if ((ab & fsel(self_sel(dy), self_sel(dx))) && ((b >> 16) & fsel(nbr_sel(dy), nbr_sel(dx))))
                            gunion(P, K, base + (a & 0xFFFFu), node_of(tn, b));
                    }
                }
            }
            // edges (-1, sy, 0)
            for (int s = -1; s <= 1; s += 2) {
                const int jy = ti.iy + s;
                if (jy < 0 || jy >= g.nt[1] || g.tblk[1][jy] != g.tblk[1][ti.iy]) continue;
                const int64_t te = tn + s * sy;
                const int lyn = g.tlen[1][jy];
                const int cyo = s < 0 ? 0 : ncy - 1, cyn = s < 0 ? (lyn - 1) / 2 : 0;
                const int jo = s < 0 ? 0 : (ti.ly - 1) & 1, jn = s < 0 ? (lyn - 1) & 1 : 0;
                const u32* FE = FACES + te * FACE_STRIDE;
                for (int cx = tid; cx < ncx; cx += NTHREADS) {
                    const u32 a = F[F_ZLO + cyo * CX + cx];
                    if (!a) continue;
                    for (int dx = -1; dx <= 1; ++dx) {
                        const int nx = cx + dx;
                        if (nx < 0 || nx >= ncx) continue;
                        const u32 b = FE[F_ZHI + cyn * CX + nx];
                        if (!b) continue;
                        if (((a >> 16) & fsel(jo, self_sel(dx))) && ((b >> 16) & fsel(jn, nbr_sel(dx))))
                            gunion(P, K, base + (a & 0xFFFFu), node_of(te, b));
                    }
                }
            }
            // edges (-1, 0, sx)
            for (int s = -1; s <= 1; s += 2) {
                const int jx = ti.ix + s;
                if (jx < 0 || jx >= g.nt[2] || g.tblk[2][jx] != g.tblk[2][ti.ix]) continue;
                const int64_t te = tn + s;
                const int lxn = g.tlen[2][jx];
                const int cxo = s < 0 ? 0 : ncx - 1, cxn = s < 0 ? (lxn - 1) / 2 : 0;
                const int io = s < 0 ? 0 : (ti.lx - 1) & 1, in_ = s < 0 ? (lxn - 1) & 1 : 0;
                const u32* FE = FACES + te * FACE_STRIDE;
                for (int cy = tid; cy < ncy; cy += NTHREADS) {
                    const u32 a = F[F_ZLO + cy * CX + cxo];
                    if (!a) continue;
                    for (int dy = -1; dy <= 1; ++dy) {
                        const int ny = cy + dy;
                        if (ny < 0 || ny >= ncy) continue;
                        const u32 b = FE[F_ZHI + ny * CX + cxn];
                        if (!b) continue;
                        if (((a >> 16) & fsel(self_sel(dy), io)) && ((b >> 16) & fsel(nbr_sel(dy), in_)))
                            gunion(P, K, base + (a & 0xFFFFu), node_of(te, b));
                    }
                }
            }
            // corners (-1, sy, sx)
            if (tid < 4) {
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
                    const u32 a = F[F_ZLO + cyo * CX + cxo];
                    const u32 b = FACES[tc * FACE_STRIDE + F_ZHI + cyn * CX + cxn];
                    if (a && b && ((a >> 16) & fsel(jo, io)) && ((b >> 16) & fsel(jn, in_)))
                        gunion(P, K, base + (a & 0xFFFFu), node_of(tc, b));
                }
            }
        }
    }
    // ---------------- y-lower seam ----------------
    if (ti.iy > 0) {
        const bool same_y = g.tblk[1][ti.iy] == g.tblk[1][ti.iy - 1];
        const int64_t tn = t - sy;
        const u32* FN = FACES + tn * FACE_STRIDE;
        if (INTER) {
            if (!same_y)
                for (int e = tid; e < ncz * CX; e += NTHREADS) {
                    const int cx = e % CX;
                    if (cx >= ncx) continue;
                    const u32 a = F[F_YLO + e];
                    if (!a) continue;
                    const u32 b = FN[F_YHI + e];
                    if ((a >> 16) & (b >> 16)) gunion(P, K, base + (a & 0xFFFFu), node_of(tn, b));
                }
        } else if (same_y) {
            // face (0, -1, 0): offsets (dz, dx)
            for (int e = tid; e < ncz * CX; e += NTHREADS) {
                const int cz = e / CX, cx = e % CX;
                if (cx >= ncx) continue;
                const u32 a = F[F_YLO + e];
                if (!a) continue;
                for (int dz = -1; dz <= 1; ++dz) {
                    const int nz = cz + dz;
                    if (nz < 0 || nz >= ncz) continue;
                    for (int dx = -1; dx <= 1; ++dx) {
                        const int nx = cx + dx;
                        if (nx < 0 || nx >= ncx) continue;
                        const u32 b = FN[F_YHI + nz * CX + nx];
                        if (!b) continue;
                        if (((a >> 16) & fsel(self_sel(dz), self_sel(dx))) && ((b >> 16) & fsel(nbr_sel(dz), nbr_sel(dx))))
                            gunion(P, K, base + (a & 0xFFFFu), node_of(tn, b));
                    }
                }
            }
            // edges (0, -1, sx)
            for (int s = -1; s <= 1; s += 2) {
                const int jx = ti.ix + s;
                if (jx < 0 || jx >= g.nt[2] || g.tblk[2][jx] != g.tblk[2][ti.ix]) continue;
                const int64_t te = tn + s;
                const int lxn = g.tlen[2][jx];
                const int cxo = s < 0 ? 0 : ncx - 1, cxn = s < 0 ? (lxn - 1) / 2 : 0;
                const int io = s < 0 ? 0 : (ti.lx - 1) & 1, in_ = s < 0 ? (lxn - 1) & 1 : 0;
                const u32* FE = FACES + te * FACE_STRIDE;
                for (int cz = tid; cz < ncz; cz += NTHREADS) {
                    const u32 a = F[F_YLO + cz * CX + cxo];
                    if (!a) continue;
                    for (int dz = -1; dz <= 1; ++dz) {
                        const int nz = cz + dz;
                        if (nz < 0 || nz >= ncz) continue;
                        const u32 b = FE[F_YHI + nz * CX + cxn];
                        if (!b) continue;
                        if (((a >> 16) & fsel(self_sel(dz), io)) && ((b >> 16) & fsel(nbr_sel(dz), in_)))
                            gunion(P, K, base + (a & 0xFFFFu), node_of(te, b));
                    }
                }
            }
        }
    }
    // ---------------- x-lower seam ----------------
    if (ti.ix > 0) {
        const bool same_x = g.tblk[2][ti.ix] == g.tblk[2][ti.ix - 1];
        const int64_t tn = t - 1;
        const u32* FN = FACES + tn * FACE_STRIDE;
        if (INTER) {
            if (!same_x)
                for (int e = tid; e < ncz * CY; e += NTHREADS) {
                    const int cy = e % CY;
                    if (cy >= ncy) continue;
                    const u32 a = F[F_XLO + e];
                    if (!a) continue;
                    const u32 b = FN[F_XHI + e];
                    if ((a >> 16) & (b >> 16)) gunion(P, K, base + (a & 0xFFFFu), node_of(tn, b));
                }
        } else if (same_x) {
            for (int e = tid; e < ncz * CY; e += NTHREADS) {
                const int cz = e / CY, cy = e % CY;
                if (cy >= ncy) continue;
                const u32 a = F[F_XLO + e];
                if (!a) continue;
                for (int dz = -1; dz <= 1; ++dz) {
                    const int nz = cz + dz;
                    if (nz < 0 || nz >= ncz) continue;
                    for (int dy = -1; dy <= 1; ++dy) {
                        const int ny = cy + dy;
                        if (ny < 0 || ny >= ncy) continue;
                        const u32 b = FN[F_XHI + nz * CY + ny];
                        if (!b) continue;
                        if (((a >> 16) & fsel(self_sel(dz), self_sel(dy))) && ((b >> 16) & fsel(nbr_sel(dz), nbr_sel(dy))))
                            gunion(P, K, base + (a & 0xFFFFu), node_of(tn, b));
                    }
                }
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// block-local roots -> sort keys
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(NTHREADS) void k_collect_roots(Geom g, const u32* COUNT, u32* P, const u64* KEY,
                                                            u64* keys, u32* vals, u32* counter) {
    const int64_t t = blockIdx.x;
    const u32 R = COUNT[t];
    if (R == 0) return;
    const TileInfo ti = tile_info(g, t);
    const u32 base = (u32)(t * g.cap);
    for (u32 k = threadIdx.x; k < R; k += NTHREADS) {
        const u32 node = base + k;
        if (P[node] == node) {
            const u32 pos = atomicAdd(counter, 1u);
            keys[pos] = ((u64)ti.block << KEY_BITS) | KEY[node];
            vals[pos] = node;
        }
    }
}

__global__ __launch_bounds__(NTHREADS) void k_count_roots(Geom g, const u32* COUNT, u32* P, u32* counter) {
    const int64_t t = blockIdx.x;
    const u32 R = COUNT[t];
    if (R == 0) return;
    const u32 base = (u32)(t * g.cap);
    u32 n = 0;
    for (u32 k = threadIdx.x; k < R; k += NTHREADS) n += (P[base + k] == base + k);
    if (n) atomicAdd(counter, n);
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

__global__ void k_nlabels(int64_t nb, const u64* values, const u64* offsets, u64* scalars) {
    if (threadIdx.x == 0 && blockIdx.x == 0) scalars[0] = offsets[nb - 1] + values[nb - 1] + 1;  // merge_offsets.py:120
}

__global__ void k_assign_rid(int64_t n, const u64* keys, const u32* vals, const u32* seg_start,
                             const u64* offsets, u64* KR) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const u64 b = keys[i] >> KEY_BITS;
    KR[vals[i]] = offsets[b] + (u64)(i - seg_start[b]) + 1;   // skimage label = rank + 1
}

__global__ void k_lut_init(u64 cap, const u64* scalars, u64* lut) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < cap && i < scalars[0]) lut[i] = i;
}

__global__ void k_lut(int64_t n, const u32* vals, u32* P, const u64* KR, u64* lut, u64* scalars) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const u32 node = vals[i];
    const u32 r = gfind(P, node);
    lut[KR[node]] = KR[r];
    if (r == node) atomicAdd((unsigned long long*)&scalars[1], 1ull);   // distinct components
}

// final label of every node.  FIN may alias KR when !LOCAL: roots keep their rid, so a
// concurrent reader of a root's entry never sees an overwritten value.  LOCAL (stage-level
// block_components) writes the block-local skimage label rid - offset into a separate FIN.
template <bool LOCAL>
__global__ __launch_bounds__(NTHREADS) void k_finalize(Geom g, const u32* COUNT, u32* P, const u64* KR,
                                                       const u64* offsets, u64* FIN) {
    const int64_t t = blockIdx.x;
    const u32 R = COUNT[t];
    if (R == 0) return;
    const u32 base = (u32)(t * g.cap);
    u64 off = 0;
    if (LOCAL) off = offsets[tile_info(g, t).block];
    for (u32 k = threadIdx.x; k < R; k += NTHREADS) {
        const u32 node = base + k;
        const u64 v = KR[gfind(P, node)];
        FIN[node] = LOCAL ? v - off : v;
    }
}

// ------------------------------------------------------------------------------------------
// k_pass2: recompute the tile CCL from the bit rows and write the uint64 labels
// ------------------------------------------------------------------------------------------
constexpr int LABCAP = 1024;

__global__ __launch_bounds__(NTHREADS) void k_pass2(Geom g, const u64* __restrict__ BITS, const u32* COUNT,
                                                    const u64* __restrict__ FIN, u64* __restrict__ out) {
    __shared__ u64 rows[NROWS];
    __shared__ u8 cm[NC];
    __shared__ u32 par[NC];
    __shared__ u64 lab[LABCAP];
    __shared__ u32 scratch[8];
    const int64_t t = blockIdx.x;
    const TileInfo ti = tile_info(g, t);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const u32 R = COUNT[t];
    const int nrows = ti.lz * ti.ly;
    const bool act = lane < ti.lx;
    if (R == 0) {
        for (int r = wave; r < nrows; r += NTHREADS / 64) {
            const int z = ti.z0 + r / ti.ly, y = ti.y0 + r % ti.ly;
            if (act) out[((int64_t)z * g.Y + y) * g.X + ti.x0 + lane] = 0;
        }
        return;
    }
    for (int i = tid; i < NROWS; i += NTHREADS) rows[i] = BITS[t * NROWS + i];
    __syncthreads();
    tile_ccl(rows, cm, par, scratch);
    const u32 base = (u32)(t * g.cap);
    for (u32 k = tid; k < R && k < LABCAP; k += NTHREADS) lab[k] = FIN[base + k];
    __syncthreads();
    for (int r = wave; r < nrows; r += NTHREADS / 64) {
        const int lzz = r / ti.ly, lyy = r % ti.ly;
        const u64 bits = rows[lzz * TY + lyy];
        if (!act) continue;
        u64 v = 0;
        if ((bits >> lane) & 1) {
            const u32 k = cube_k(par, ((lzz >> 1) * CY + (lyy >> 1)) * CX + (lane >> 1));
            v = k < LABCAP ? lab[k] : FIN[base + k];
        }
        out[((int64_t)(ti.z0 + lzz) * g.Y + ti.y0 + lyy) * g.X + ti.x0 + lane] = v;
    }
}

// instantiate the templates used by the host side
template __global__ void k_pass1<false>(Geom, const float*, const u8*, const BlockParam*, float, int, u64*, u32*, u32*, u32*, u64*);
template __global__ void k_pass1<true>(Geom, const float*, const u8*, const BlockParam*, float, int, u64*, u32*, u32*, u32*, u64*);
template __global__ void k_stitch<false>(Geom, const u32*, u32*, const u64*);
template __global__ void k_stitch<true>(Geom, const u32*, u32*, const u64*);
template __global__ void k_finalize<false>(Geom, const u32*, u32*, const u64*, const u64*, u64*);
template __global__ void k_finalize<true>(Geom, const u32*, u32*, const u64*, const u64*, u64*);

}  // namespace cc
