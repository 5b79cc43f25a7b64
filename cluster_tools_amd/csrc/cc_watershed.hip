// cc_watershed.hip -- seeded watershed per block (§8f, the other half of rank 4): the reference's
// WatershedFromSeeds task (watershed/watershed_from_seeds.py:143-273, used by
// ThresholdAndWatershedWorkflow, thresholded_components_workflow.py:107-144) grows the
// thresholded components (the seeds) over the normalized input, block by block without halo,
// through `vu.watershed(input_, seeds, size_filter)` -- a function the reference's volume_utils
// does not define, so there is no behaviour to pin (parity UNPINNED; oracle/watershed.py
// restates the definition below and is what the tests check against).
//
// Definition (per block of the reference blocking, 6-connected inside the block):
//   f(v)     = vu.normalize of the block (float32 (x - min) / max(x - min), volume_utils.py:98-105),
//              1.0 outside the mask (_ws_block_masked), as an ordered u32; NaN -> 0xFFFFFFFE
//   cost(v)  = 0 for seeds, else the min over paths from a seed of the max f on the path (the
//              seed excluded): the least fixpoint of cost(v) = min_u max(cost(u), f(v))
//   label(v) = the seed's id for seeds, else the smallest label among the 6-neighbours u with
//              max(cost(u), f(v)) == cost(v) (the neighbours an optimal path can come through),
//              i.e. the smallest seed label reaching v in that predecessor graph; 0 where no
//              seed reaches v (a block without seeds) and outside the mask.
// Both fixpoints are unique (min over a fixed, monotone system), so any update order reaches
// them: here tiles of 8 x 8 x 32 voxels (inside one block) relax in LDS to their local fixpoint
// given the halo (voxel-by-voxel sweeps), rounds of launches over the tiles whose neighbours
// changed until none changes (phase 1: costs; phase 2: labels on the converged costs).  Every
// round after a phase's first visits only the tiles the previous round listed.
namespace cc {

// tile shape and threads (CC_WS_TZ / TY / TX / TT at build time, each on its own: A/B only)
#ifndef CC_WS_TZ
#define CC_WS_TZ 8
#endif
#ifndef CC_WS_TY
#define CC_WS_TY 8
#endif
#ifndef CC_WS_TX
#define CC_WS_TX 32
#endif
#ifndef CC_WS_TT
#define CC_WS_TT 256
#endif
constexpr int WS_Z = CC_WS_TZ, WS_Y = CC_WS_TY, WS_X = CC_WS_TX, WS_T = CC_WS_TT;
static_assert(WS_Z * WS_Y * WS_X % WS_T == 0, "whole voxels per thread");
static_assert(WS_T % 64 == 0 && WS_T >= 64, "whole waves per tile");
static_assert(WS_T >= 6, "ws_list_neighbours lists the six face neighbours with one thread each");
#ifndef CC_WS_ALT
#define CC_WS_ALT 0        // A/B only: odd sweeps walk a thread's voxels in reverse order
#endif
constexpr int WS_HZ = WS_Z + 2, WS_HY = WS_Y + 2, WS_HX = WS_X + 2, WS_HN = WS_HZ * WS_HY * WS_HX;
constexpr int WS_VPT = WS_Z * WS_Y * WS_X / WS_T;      // interior voxels per thread
constexpr u32 WS_INF = 0xFFFFFFFFu;

struct WsGeom {
    int64_t S[3], B[3];           // volume and block shape
    int32_t nt[3], nb[3];         // watershed tiles / blocks per axis
    const int32_t* tstart[3];     // per-axis tile tables (tiles tiled from each block's origin)
    const int32_t* tlen[3];
    const int32_t* tblk[3];
};

// ordered f of one voxel (see the definition above)
__device__ __forceinline__ u32 ws_f(float x, float mn, float m, bool nan, bool in_mask) {
    float y = 1.0f;
    if (in_mask) {
        y = x - mn;
        if (m > 0.0f) y = y / m;
    }
    const u32 b = __float_as_uint(y);
    if ((in_mask && nan) || (b & 0x7FFFFFFFu) > 0x7F800000u) return 0xFFFFFFFEu;
    return f2ord(b);
}

__global__ void k_fill_u32(int64_t n, u32* p, u32 v) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

__global__ void k_ws_init(int64_t n, const u64* __restrict__ seeds, u32* cost, u32* lab, u32* err) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const u64 s = seeds[i];
        if (s >= (u64)WS_INF) atomicOr(err, 1u);
        cost[i] = s ? 0u : WS_INF;
        lab[i] = s ? (u32)s : WS_INF;
    }
}

// a watershed tile: position, extent, block and the block's extent (neighbours outside the block
// are not neighbours: blocks are independent)
struct WsTile {
    int ix, iy, iz, z0, y0, x0, lz, ly, lx, bz, by, bx;
    int64_t b, e0[3], e1[3];
};

__device__ __forceinline__ WsTile ws_tile(const WsGeom& g, int64_t t) {
    WsTile w;
    const u32 tt = (u32)t, n2 = (u32)g.nt[2], n1 = (u32)g.nt[1];
    const u32 q = tt / n2;
    w.ix = (int)(tt - q * n2); w.iy = (int)(q % n1); w.iz = (int)(q / n1);
    w.z0 = g.tstart[0][w.iz]; w.y0 = g.tstart[1][w.iy]; w.x0 = g.tstart[2][w.ix];
    w.lz = g.tlen[0][w.iz]; w.ly = g.tlen[1][w.iy]; w.lx = g.tlen[2][w.ix];
    w.bz = g.tblk[0][w.iz]; w.by = g.tblk[1][w.iy]; w.bx = g.tblk[2][w.ix];
    w.b = ((int64_t)w.bz * g.nb[1] + w.by) * g.nb[2] + w.bx;
    w.e0[0] = w.bz * g.B[0]; w.e0[1] = w.by * g.B[1]; w.e0[2] = w.bx * g.B[2];
#pragma unroll
    for (int a = 0; a < 3; ++a) w.e1[a] = w.e0[a] + g.B[a] < g.S[a] ? w.e0[a] + g.B[a] : g.S[a];
    return w;
}

// the tile's state with its halo into LDS (WS_INF outside the block)
__device__ __forceinline__ void ws_load_halo(const WsGeom& g, const WsTile& w, const u32* __restrict__ src, u32* H) {
    const int64_t YX = g.S[1] * g.S[2];
    for (int i = threadIdx.x; i < WS_HN; i += WS_T) {
        const int hz = i / (WS_HY * WS_HX), hy = (i / WS_HX) % WS_HY, hx = i % WS_HX;
        const int64_t z = w.z0 - 1 + hz, y = w.y0 - 1 + hy, x = w.x0 - 1 + hx;
        const bool inside_tile = hz >= 1 && hy >= 1 && hx >= 1 && hz <= w.lz && hy <= w.ly && hx <= w.lx;
        const bool halo = !inside_tile && z >= w.e0[0] && z < w.e1[0] && y >= w.e0[1] && y < w.e1[1] &&
                          x >= w.e0[2] && x < w.e1[2];
        H[i] = (inside_tile || halo) ? src[z * YX + y * g.S[2] + x] : WS_INF;
    }
}

// the six neighbour tiles of the same block see a new halo: each goes on the next round's list
// once (stamp = the round that listed it)
__device__ __forceinline__ void ws_list_neighbours(const WsGeom& g, const WsTile& w, int64_t t, u32* stamp, u32 round,
                                                   u32* list_out, u32* n_out) {
    const int tid = threadIdx.x;
    if (tid >= 6) return;
    const int64_t n2 = g.nt[2], zs = (int64_t)g.nt[1] * n2;
    bool ok = false;
    int64_t u = 0;
    switch (tid) {
        case 0: ok = w.iz > 0 && g.tblk[0][w.iz - 1] == w.bz; u = t - zs; break;
        case 1: ok = w.iz + 1 < g.nt[0] && g.tblk[0][w.iz + 1] == w.bz; u = t + zs; break;
        case 2: ok = w.iy > 0 && g.tblk[1][w.iy - 1] == w.by; u = t - n2; break;
        case 3: ok = w.iy + 1 < g.nt[1] && g.tblk[1][w.iy + 1] == w.by; u = t + n2; break;
        case 4: ok = w.ix > 0 && g.tblk[2][w.ix - 1] == w.bx; u = t - 1; break;
        default: ok = w.ix + 1 < g.nt[2] && g.tblk[2][w.ix + 1] == w.bx; u = t + 1; break;
    }
    if (ok && atomicExch(&stamp[u], round) != round) list_out[atomicAdd(n_out, 1u)] = (u32)u;
}

constexpr int WS_DZ = WS_HY * WS_HX, WS_DY = WS_HX;

// label sweeps over the predecessor masks (bit d: the neighbour in direction d, in the order
// -z, +z, -y, +y, -x, +x, is an optimal predecessor) to the tile's fixpoint; true if any changed
__device__ __forceinline__ bool ws_label_sweeps(const WsTile& w, u32* L, const u8* PM) {
    const int tid = threadIdx.x;
    bool tile_changed = false;
    for (int sweep = 0;; ++sweep) {
        bool chg = false;
#pragma unroll
        for (int k = 0; k < WS_VPT; ++k) {
            const int j = tid + (CC_WS_ALT && (sweep & 1) ? WS_VPT - 1 - k : k) * WS_T;
            const u32 pm = PM[j];
            if (!pm) continue;
            const int vz = j / (WS_Y * WS_X), vy = (j / WS_X) % WS_Y, vx = j % WS_X;
            const int h = ((vz + 1) * WS_HY + vy + 1) * WS_HX + vx + 1;
            u32 l = L[h];
            const u32 l0 = l;
            if (pm & 1u) l = min(l, L[h - WS_DZ]);
            if (pm & 2u) l = min(l, L[h + WS_DZ]);
            if (pm & 4u) l = min(l, L[h - WS_DY]);
            if (pm & 8u) l = min(l, L[h + WS_DY]);
            if (pm & 16u) l = min(l, L[h - 1]);
            if (pm & 32u) l = min(l, L[h + 1]);
            if (l < l0) { L[h] = l; chg = true; }
        }
        if (!__syncthreads_or(chg)) break;
        tile_changed = true;
    }
    return tile_changed;
}

__device__ __forceinline__ void ws_store(const WsGeom& g, const WsTile& w, const u32* H, u32* dst) {
    const int64_t YX = g.S[1] * g.S[2];
    for (int j = threadIdx.x; j < WS_Z * WS_Y * WS_X; j += WS_T) {
        const int vz = j / (WS_Y * WS_X), vy = (j / WS_X) % WS_Y, vx = j % WS_X;
        if (vz >= w.lz || vy >= w.ly || vx >= w.lx) continue;
        const int h = ((vz + 1) * WS_HY + vy + 1) * WS_HX + vx + 1;
        dst[(int64_t)(w.z0 + vz) * YX + (int64_t)(w.y0 + vy) * g.S[2] + (w.x0 + vx)] = H[h];
    }
}

// PHASE 1: one round of the costs over the round's tiles.  PHASE 2: every tile once on the
// converged costs: each voxel's predecessor mask (pm), which is all the label rounds (k_ws_label)
// read besides the labels (half their LDS, twice the resident tiles).
template <int PHASE>
__global__ __launch_bounds__(WS_T) void k_ws_relax(WsGeom g, const float* __restrict__ in, const u8* __restrict__ mask,
                                                   const u32* __restrict__ smin, const u32* __restrict__ smax,
                                                   const u32* __restrict__ sflag, u32* cost, u32* lab, u8* pm,
                                                   const u32* __restrict__ list_in, u32* stamp, u32 round,
                                                   u32* list_out, u32* n_out) {
    __shared__ u32 C[WS_HN], F[WS_Z * WS_Y * WS_X];
    // the round's tiles: all (list_in NULL, the first round of a phase) or the listed ones
    const int64_t t = list_in ? (int64_t)list_in[blockIdx.x] : (int64_t)blockIdx.x;
    const int tid = threadIdx.x;
    const WsTile w = ws_tile(g, t);
    // normalize parameters of the block (as block_param: numpy's min / max(x - min), NaN blocks)
    const u32 omn = smin[w.b], omx = smax[w.b];
    const bool nan = sflag[w.b] & 1u;
    const float mn = __uint_as_float(ord2f(omn)), mxv = __uint_as_float(ord2f(omx));
    const float m = (isinf(mn) || isinf(mxv)) ? (isinf(mn) ? __uint_as_float(0x7FC00000u) : mxv - mn) : mxv - mn;
    const int64_t YX = g.S[1] * g.S[2];
    ws_load_halo(g, w, cost, C);
    for (int j = tid; j < WS_Z * WS_Y * WS_X; j += WS_T) {
        const int vz = j / (WS_Y * WS_X), vy = (j / WS_X) % WS_Y, vx = j % WS_X;
        u32 f = WS_INF;
        if (vz < w.lz && vy < w.ly && vx < w.lx) {
            const int64_t o = (int64_t)(w.z0 + vz) * YX + (int64_t)(w.y0 + vy) * g.S[2] + (w.x0 + vx);
            f = ws_f(in[o], mn, m, nan, mask == nullptr || mask[o] != 0);
        }
        F[j] = f;
    }
    __syncthreads();
    bool tile_changed = false;
    if (PHASE == 1) {
        // voxel-by-voxel (Gauss-Seidel) sweeps: each voxel against its six neighbours
        for (int sweep = 0;; ++sweep) {
            bool chg = false;
#pragma unroll
            for (int k = 0; k < WS_VPT; ++k) {
                const int j = tid + (CC_WS_ALT && (sweep & 1) ? WS_VPT - 1 - k : k) * WS_T;
                const int vz = j / (WS_Y * WS_X), vy = (j / WS_X) % WS_Y, vx = j % WS_X;
                if (vz >= w.lz || vy >= w.ly || vx >= w.lx) continue;
                const int h = ((vz + 1) * WS_HY + vy + 1) * WS_HX + vx + 1;
                const u32 c = C[h];
                if (c == 0u) continue;                               // a seed
                const u32 best = min(min(min(C[h - WS_DZ], C[h + WS_DZ]), min(C[h - WS_DY], C[h + WS_DY])),
                                     min(C[h - 1], C[h + 1]));
                const u32 cand = best == WS_INF ? WS_INF : max(best, F[j]);
                if (cand < c) { C[h] = cand; chg = true; }
            }
            if (!__syncthreads_or(chg)) break;
            tile_changed = true;
        }
        if (tile_changed) ws_store(g, w, C, cost);
    } else {
        for (int j = tid; j < WS_Z * WS_Y * WS_X; j += WS_T) {
            const int vz = j / (WS_Y * WS_X), vy = (j / WS_X) % WS_Y, vx = j % WS_X;
            if (vz >= w.lz || vy >= w.ly || vx >= w.lx) continue;
            const int h = ((vz + 1) * WS_HY + vy + 1) * WS_HX + vx + 1;
            const u32 c = C[h], f = F[j];
            u32 bits = 0;
            if (c != 0u && c != WS_INF) {
                const int off[6] = {-WS_DZ, WS_DZ, -WS_DY, WS_DY, -1, 1};
#pragma unroll
                for (int d = 0; d < 6; ++d) {
                    const u32 cu = C[h + off[d]];
                    if (cu != WS_INF && max(cu, f) == c) bits |= 1u << d;
                }
            }
                pm[(int64_t)(w.z0 + vz) * YX + (int64_t)(w.y0 + vy) * g.S[2] + (w.x0 + vx)] = (u8)bits;
        }
        return;                                       // the label rounds are k_ws_label's
    }
    if (tile_changed) ws_list_neighbours(g, w, t, stamp, round, list_out, n_out);
}

// a label round over the listed tiles (list_in NULL: every tile): labels with halo and the
// predecessor masks
__global__ __launch_bounds__(WS_T) void k_ws_label(WsGeom g, const u8* __restrict__ pm, u32* lab,
                                                   const u32* __restrict__ list_in, u32* stamp, u32 round,
                                                   u32* list_out, u32* n_out) {
    __shared__ u32 Lsh[WS_HN];
    __shared__ u8 PM[WS_Z * WS_Y * WS_X];
    const int64_t t = list_in ? (int64_t)list_in[blockIdx.x] : (int64_t)blockIdx.x;
    const WsTile w = ws_tile(g, t);
    const int64_t YX = g.S[1] * g.S[2];
    ws_load_halo(g, w, lab, Lsh);
    for (int j = threadIdx.x; j < WS_Z * WS_Y * WS_X; j += WS_T) {
        const int vz = j / (WS_Y * WS_X), vy = (j / WS_X) % WS_Y, vx = j % WS_X;
        u8 bits = 0;
        if (vz < w.lz && vy < w.ly && vx < w.lx)
            bits = pm[(int64_t)(w.z0 + vz) * YX + (int64_t)(w.y0 + vy) * g.S[2] + (w.x0 + vx)];
        PM[j] = bits;
    }
    __syncthreads();
    if (ws_label_sweeps(w, Lsh, PM)) {
        ws_store(g, w, Lsh, lab);
        ws_list_neighbours(g, w, t, stamp, round, list_out, n_out);
    }
}

__global__ void k_ws_write(int64_t n, const u32* __restrict__ lab, const u8* __restrict__ mask, u64* out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const u32 l = lab[i];
        out[i] = (l == WS_INF || (mask && !mask[i])) ? 0ull : (u64)l;
    }
}

// ---- 4-D (channel) input of the watershed (_read_data, watershed_from_seeds.py:127-139): the
// selected channels of the (C, Z, Y, X) block are normalized together (vu.normalize of the 4-D
// block: one min / max over every channel of the block), then aggregated over the channels by
// np.mean / np.max / np.min(axis=0) in channel order (float32; mean: sequential sum, then / C).
// Per block: (mn, m) as block_param derives them; NaN blocks -> NaN everywhere (x - NaN).
__global__ void k_norm_params(int64_t nb, const u32* smin, const u32* smax, const u32* sflag, float2* nm) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    float mn = __uint_as_float(ord2f(smin[b]));
    const float mx = __uint_as_float(ord2f(smax[b]));
    float m = isinf(mn) ? __uint_as_float(0x7FC00000u) : mx - mn;     // numpy: (x - mn).max()
    if (sflag[b] & 1u) { mn = __uint_as_float(0x7FC00000u); m = mn; }  // NaN: x.min() is NaN
    nm[b] = make_float2(mn, m);
}

template <int AGG>   // 0 mean, 1 max, 2 min
__global__ void k_norm_agg(const float* __restrict__ in, int nc, int64_t Z, int64_t Y, int64_t X, int64_t Bz, int64_t By,
                           int64_t Bx, int nby, int nbx, const float2* __restrict__ nm, float* __restrict__ out) {
    const int64_t n = Z * Y * X;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t x = i % X, y = (i / X) % Y, z = i / (X * Y);
        const float2 p = nm[((z / Bz) * nby + y / By) * nbx + x / Bx];
        float acc = 0.0f;
        for (int c = 0; c < nc; ++c) {
            float v = __fsub_rn(in[(int64_t)c * n + i], p.x);          // vu.normalize, no contraction
            if (p.y > 0.0f) v = __fdiv_rn(v, p.y);
            if (c == 0) acc = v;
            else if (AGG == 0) acc = __fadd_rn(acc, v);
            else if (AGG == 1) acc = (acc >= v || isnan(acc)) ? acc : v;    // np.maximum: NaN propagates
            else acc = (acc <= v || isnan(acc)) ? acc : v;                  // np.minimum
        }
        out[i] = AGG == 0 ? __fdiv_rn(acc, (float)nc) : acc;
    }
}

// The same per voxel row: one workgroup per (z, y) row, float4 per lane (X and the block's x
// extent multiples of 4, so a float4 never straddles two blocks); the block lookup per float4 and
// no per-voxel 64-bit index arithmetic (the element kernel above spent its time there: 21.8 ms
// for three C3 channels = 3.2 TB/s, profiles/r04_misc_summary.txt).
template <int AGG>
__global__ __launch_bounds__(256) void k_norm_agg4(const float* __restrict__ in, int nc, int64_t Y, int64_t X,
                                                   int64_t Bz, int64_t By, int Bx, int nby, int nbx,
                                                   const float2* __restrict__ nm, float* __restrict__ out, int64_t n) {
    const int64_t r = blockIdx.x;                    // row z * Y + y
    const int64_t z = r / Y, y = r - z * Y;
    const int64_t brow = ((z / Bz) * nby + y / By) * nbx;
    const int x4n = (int)(X / 4);
    for (int x4 = threadIdx.x; x4 < x4n; x4 += 256) {
        const float2 p = nm[brow + (4 * x4) / Bx];
        const int64_t i = r * X + 4 * x4;
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int c = 0; c < nc; ++c) {
            const float4 u = *reinterpret_cast<const float4*>(in + (int64_t)c * n + i);
            float v[4] = {__fsub_rn(u.x, p.x), __fsub_rn(u.y, p.x), __fsub_rn(u.z, p.x), __fsub_rn(u.w, p.x)};
            float* a = &acc.x;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if (p.y > 0.0f) v[e] = __fdiv_rn(v[e], p.y);
                if (c == 0) a[e] = v[e];
                else if (AGG == 0) a[e] = __fadd_rn(a[e], v[e]);
                else if (AGG == 1) a[e] = (a[e] >= v[e] || isnan(a[e])) ? a[e] : v[e];
                else a[e] = (a[e] <= v[e] || isnan(a[e])) ? a[e] : v[e];
            }
        }
        if (AGG == 0) {
            const float d = (float)nc;
            acc = make_float4(__fdiv_rn(acc.x, d), __fdiv_rn(acc.y, d), __fdiv_rn(acc.z, d), __fdiv_rn(acc.w, d));
        }
        *reinterpret_cast<float4*>(out + i) = acc;
    }
}

}  // namespace cc

extern "C" int cc_normalize_channels(cc_ctx* c, const float* in, int64_t n_channels, const int64_t shape[3],
                                     const int64_t block_shape[3], int agg, float* out) {
    CC_TRY({
        CC_REQUIRE(c && in && out && shape && block_shape, "NULL argument");
        require_row_aligned(in, shape[2] * 4);
        require_row_aligned(out, shape[2] * 4);
        CC_REQUIRE(n_channels >= 1 && n_channels < (1 << 20), "need at least one channel");
        CC_REQUIRE(agg >= 0 && agg <= 2, "agg must be 0 (mean), 1 (max) or 2 (min)");
        HIP_OK(hipSetDevice(c->device));
        hipStream_t s = cstream(c);
        RunState& st = state(c);
        st = RunState();
        st.hg = make_geom(shape, block_shape, 0);
        upload_geom(c, st.hg);
        Geom& gg = st.hg.g;
        const int64_t nb = gg.n_blocks, n = shape[0] * shape[1] * shape[2];
        c->bstat.ensure(nb * 3 * sizeof(u32));
        u32* smin = c->bstat.as<u32>();
        u32* smax = smin + nb;
        u32* sflag = smax + nb;
        HIP_OK(hipMemsetAsync(smin, 0xFF, nb * sizeof(u32), s));
        HIP_OK(hipMemsetAsync(smax, 0x00, 2 * nb * sizeof(u32), s));
        // the 4-D block's min / max: every channel's tiles fold into the same block statistics
        for (int64_t ch = 0; ch < n_channels; ++ch)
            launch(c, "k_block_stats", [&] { k_block_stats<<<(unsigned)gg.n_tiles, NTHREADS, 0, s>>>(gg, in + ch * n, smin, smax, sflag); });
        c->gs_tab.ensure(nb * sizeof(float2));
        float2* nm = c->gs_tab.as<float2>();
        launch(c, "k_norm_params", [&] { k_norm_params<<<grid1d(nb), 256, 0, s>>>(nb, smin, smax, sflag, nm); });
        const int nby = gg.nb[1], nbx = gg.nb[2];
        const bool rows4 = shape[2] % 4 == 0 && block_shape[2] % 4 == 0 && block_shape[2] < (1LL << 31) &&
                           ((uintptr_t)in | (uintptr_t)out) % 16 == 0 && shape[0] * shape[1] < (1LL << 31);
        launch(c, "k_norm_agg", [&] {
            auto run = [&](auto kern) {
                kern<<<grid_stride(n), 256, 0, s>>>(in, (int)n_channels, shape[0], shape[1], shape[2], block_shape[0],
                                                   block_shape[1], block_shape[2], nby, nbx, nm, out);
            };
            auto run4 = [&](auto kern) {
                kern<<<(unsigned)(shape[0] * shape[1]), 256, 0, s>>>(in, (int)n_channels, shape[1], shape[2], block_shape[0],
                                                                    block_shape[1], (int)block_shape[2], nby, nbx, nm, out, n);
            };
            if (rows4) {
                if (agg == 0) run4(k_norm_agg4<0>);
                else if (agg == 1) run4(k_norm_agg4<1>);
                else run4(k_norm_agg4<2>);
            } else if (agg == 0) run(k_norm_agg<0>);
            else if (agg == 1) run(k_norm_agg<1>);
            else run(k_norm_agg<2>);
        });
        sync(c);
    })
}

extern "C" int cc_watershed_from_seeds(cc_ctx* c, const float* in, const uint64_t* seeds, const uint8_t* mask,
                                       const int64_t shape[3], const int64_t block_shape[3], uint64_t* out,
                                       int64_t* rounds) {
    CC_TRY({
        CC_REQUIRE(c && in && seeds && out && shape && block_shape, "NULL argument");
        require_row_aligned(in, shape[2] * 4);
        require_row_aligned(seeds, shape[2] * 8);
        require_row_aligned(mask, shape[2]);
        require_row_aligned(out, shape[2] * 8);
        HIP_OK(hipSetDevice(c->device));
        hipStream_t s = cstream(c);
        // block statistics (normalize), the labelling path's tiles
        RunState& st = state(c);
        st = RunState();
        st.hg = make_geom(shape, block_shape, 0);
        upload_geom(c, st.hg);
        Geom& gg = st.hg.g;
        const int64_t nb = gg.n_blocks, n = shape[0] * shape[1] * shape[2];
        c->bstat.ensure(nb * 3 * sizeof(u32));
        u32* smin = c->bstat.as<u32>();
        u32* smax = smin + nb;
        u32* sflag = smax + nb;
        if (c->ws_prenormalized) {
            // the input is already the normalized block (4-D input: cc_normalize_channels): min =
            // max = +0 and no NaN flag make f(v) = x - 0 = x, no division (NaN voxels stay NaN)
            HIP_OK(hipMemsetAsync(smin, 0x00, 2 * nb * sizeof(u32), s));
            launch(c, "k_fill_u32", [&] { k_fill_u32<<<grid1d(2 * nb), 256, 0, s>>>(2 * nb, smin, 0x80000000u); });
            HIP_OK(hipMemsetAsync(sflag, 0x00, nb * sizeof(u32), s));
        } else {
            HIP_OK(hipMemsetAsync(smin, 0xFF, nb * sizeof(u32), s));
            HIP_OK(hipMemsetAsync(smax, 0x00, 2 * nb * sizeof(u32), s));
            launch(c, "k_block_stats", [&] { k_block_stats<<<(unsigned)gg.n_tiles, NTHREADS, 0, s>>>(gg, in, smin, smax, sflag); });
        }
        // the watershed tiles: per axis, tiles of WS_* from each block's origin
        WsGeom g;
        std::memset(&g, 0, sizeof(g));
        const int T[3] = {WS_Z, WS_Y, WS_X};
        std::vector<int32_t> tab;
        std::vector<int32_t> st3[3], ln3[3], bk3[3];
        for (int a = 0; a < 3; ++a) {
            g.S[a] = shape[a];
            g.B[a] = block_shape[a];
            g.nb[a] = (int32_t)((shape[a] + block_shape[a] - 1) / block_shape[a]);
            for (int64_t bb = 0; bb < g.nb[a]; ++bb) {
                const int64_t b0 = bb * block_shape[a], b1 = std::min(b0 + block_shape[a], shape[a]);
                for (int64_t p = b0; p < b1; p += T[a]) {
                    st3[a].push_back((int32_t)p);
                    ln3[a].push_back((int32_t)std::min<int64_t>(T[a], b1 - p));
                    bk3[a].push_back((int32_t)bb);
                }
            }
            g.nt[a] = (int32_t)st3[a].size();
        }
        for (int a = 0; a < 3; ++a) {
            tab.insert(tab.end(), st3[a].begin(), st3[a].end());
            tab.insert(tab.end(), ln3[a].begin(), ln3[a].end());
            tab.insert(tab.end(), bk3[a].begin(), bk3[a].end());
        }
        const int64_t nt = (int64_t)g.nt[0] * g.nt[1] * g.nt[2];
        CC_REQUIRE(nt < (1LL << 31), "too many watershed tiles");
        c->ws_tab.ensure(tab.size() * sizeof(int32_t));
        HIP_OK(hipMemcpyAsync(c->ws_tab.p, tab.data(), tab.size() * sizeof(int32_t), hipMemcpyHostToDevice, s));
        {
            const int32_t* p = c->ws_tab.as<int32_t>();
            for (int a = 0; a < 3; ++a) {
                g.tstart[a] = p; p += g.nt[a];
                g.tlen[a] = p; p += g.nt[a];
                g.tblk[a] = p; p += g.nt[a];
            }
        }
        // state: cost | label per voxel; per tile the round that last listed it, two tile lists
        c->ws_buf.ensure((size_t)n * 2 * sizeof(u32) + 3 * (size_t)nt * sizeof(u32) + (size_t)n + 64);
        u32* cost = c->ws_buf.as<u32>();
        u32* lab = cost + n;
        u32* stamp = lab + n;
        u32* list0 = stamp + nt;
        u32* list1 = list0 + nt;
        u8* pm = (u8*)(list1 + nt);                   // predecessor masks (the first label round)
        c->counter.ensure(4 * sizeof(u32));
        u32* flags = c->counter.as<u32>();            // [0] seed id overflow, [1] tiles listed for the next round
        HIP_OK(hipMemsetAsync(flags, 0, 4 * sizeof(u32), s));
        HIP_OK(hipMemsetAsync(stamp, 0, nt * sizeof(u32), s));
        launch(c, "k_ws_init", [&] { k_ws_init<<<grid_stride(n), 256, 0, s>>>(n, seeds, cost, lab, flags); });
        int64_t total_rounds = 0;
        u32 round = 0;
        const bool trace = std::getenv("CC_WS_TRACE") != nullptr;
        auto tr0 = std::chrono::steady_clock::now();
        for (int phase = 1; phase <= 2; ++phase) {
            // the first round of a phase visits every tile, later rounds the tiles listed by the last
            const u32* lin = nullptr;
            int64_t ntile = nt;
            if (phase == 2)
                launch(c, "k_ws_preds", [&] {
                    k_ws_relax<2><<<(unsigned)nt, WS_T, 0, s>>>(g, in, mask, smin, smax, sflag, cost, lab, pm, nullptr,
                                                               stamp, round, list1, flags + 1);
                });
            for (int64_t r = 0; ntile > 0; ++r) {
                CC_REQUIRE(r < 4 * n + 16, "watershed did not converge");
                ++round;
                HIP_OK(hipMemsetAsync(flags + 1, 0, sizeof(u32), s));
                launch(c, phase == 1 ? "k_ws_relax_cost" : "k_ws_relax_label", [&] {
                    if (phase == 1)
                        k_ws_relax<1><<<(unsigned)ntile, WS_T, 0, s>>>(g, in, mask, smin, smax, sflag, cost, lab, pm, lin,
                                                                      stamp, round, list1, flags + 1);
                    else
                        k_ws_label<<<(unsigned)ntile, WS_T, 0, s>>>(g, pm, lab, lin, stamp, round, list1, flags + 1);
                });
                u32 fl[2] = {0, 0};
                {
                    Readback rb(c, 64);
                    rb.add(fl, flags, 2 * sizeof(u32));
                    rb.wait();
                }
                CC_REQUIRE(!(fl[0] & 1u), "seed ids must be < 2^32 - 1 (the reference casts seeds to uint32)");
                ++total_rounds;
                CC_REQUIRE(fl[1] <= (u32)nt, "watershed tile list overflow");
                std::swap(list0, list1);
                lin = list0;
                if (trace) {                          // dev hook: tiles and host ms per round
                    const auto now = std::chrono::steady_clock::now();
                    std::fprintf(stderr, "ws phase %d round %ld tiles %ld ms %.3f\n", phase, (long)r, (long)ntile,
                                 std::chrono::duration<double, std::milli>(now - tr0).count());
                    tr0 = now;
                }
                ntile = fl[1];
            }
        }
        launch(c, "k_ws_write", [&] { k_ws_write<<<grid_stride(n), 256, 0, s>>>(n, lab, mask, out); });
        sync(c);
        if (rounds) *rounds = total_rounds;
    })
}
