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

constexpr int WS_Z = 8, WS_Y = 8, WS_X = 32, WS_T = 256;
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

__global__ void k_ws_init(int64_t n, const u64* __restrict__ seeds, u32* cost, u32* lab, u32* err) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const u64 s = seeds[i];
        if (s >= (u64)WS_INF) atomicOr(err, 1u);
        cost[i] = s ? 0u : WS_INF;
        lab[i] = s ? (u32)s : WS_INF;
    }
}

// one round over the active tiles; PHASE 1 relaxes costs, PHASE 2 labels
template <int PHASE>
__global__ __launch_bounds__(WS_T) void k_ws_relax(WsGeom g, const float* __restrict__ in, const u8* __restrict__ mask,
                                                   const u32* __restrict__ smin, const u32* __restrict__ smax,
                                                   const u32* __restrict__ sflag, u32* cost, u32* lab,
                                                   const u32* __restrict__ list_in, u32* stamp, u32 round,
                                                   u32* list_out, u32* n_out) {
    __shared__ u32 C[WS_HN], F[WS_Z * WS_Y * WS_X];
    __shared__ u32 Lsh[PHASE == 2 ? WS_HN : 1];
    // the round's tiles: all (list_in NULL, the first round of a phase) or the listed ones
    const int64_t t = list_in ? (int64_t)list_in[blockIdx.x] : (int64_t)blockIdx.x;
    const int tid = threadIdx.x;
    const u32 tt = (u32)t, n2 = (u32)g.nt[2], n1 = (u32)g.nt[1];
    const u32 q = tt / n2;
    const int ix = (int)(tt - q * n2), iy = (int)(q % n1), iz = (int)(q / n1);
    const int z0 = g.tstart[0][iz], y0 = g.tstart[1][iy], x0 = g.tstart[2][ix];
    const int lz = g.tlen[0][iz], ly = g.tlen[1][iy], lx = g.tlen[2][ix];
    const int bz = g.tblk[0][iz], by = g.tblk[1][iy], bx = g.tblk[2][ix];
    const int64_t b = ((int64_t)bz * g.nb[1] + by) * g.nb[2] + bx;
    // the block's extent: neighbours outside it are not neighbours (blocks are independent)
    const int64_t e0[3] = {bz * g.B[0], by * g.B[1], bx * g.B[2]};
    int64_t e1[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) e1[a] = e0[a] + g.B[a] < g.S[a] ? e0[a] + g.B[a] : g.S[a];
    // normalize parameters of the block (as block_param: numpy's min / max(x - min), NaN blocks)
    const u32 omn = smin[b], omx = smax[b];
    const bool nan = sflag[b] & 1u;
    const float mn = __uint_as_float(ord2f(omn)), mxv = __uint_as_float(ord2f(omx));
    const float m = (isinf(mn) || isinf(mxv)) ? (isinf(mn) ? __uint_as_float(0x7FC00000u) : mxv - mn) : mxv - mn;
    const int64_t YX = g.S[1] * g.S[2];
    for (int i = tid; i < WS_HN; i += WS_T) {
        const int hz = i / (WS_HY * WS_HX), hy = (i / WS_HX) % WS_HY, hx = i % WS_HX;
        const int64_t z = z0 - 1 + hz, y = y0 - 1 + hy, x = x0 - 1 + hx;
        const bool inside_tile = hz >= 1 && hy >= 1 && hx >= 1 && hz <= lz && hy <= ly && hx <= lx;
        const bool halo = !inside_tile && z >= e0[0] && z < e1[0] && y >= e0[1] && y < e1[1] && x >= e0[2] && x < e1[2];
        u32 c = WS_INF, l = WS_INF;
        if (inside_tile || halo) {
            const int64_t o = z * YX + y * g.S[2] + x;
            c = cost[o];
            if (PHASE == 2) l = lab[o];
        }
        C[i] = c;
        if (PHASE == 2) Lsh[i] = l;
    }
    for (int j = tid; j < WS_Z * WS_Y * WS_X; j += WS_T) {
        const int vz = j / (WS_Y * WS_X), vy = (j / WS_X) % WS_Y, vx = j % WS_X;
        u32 f = WS_INF;
        if (vz < lz && vy < ly && vx < lx) {
            const int64_t o = (int64_t)(z0 + vz) * YX + (int64_t)(y0 + vy) * g.S[2] + (x0 + vx);
            f = ws_f(in[o], mn, m, nan, mask == nullptr || mask[o] != 0);
        }
        F[j] = f;
    }
    __syncthreads();
    constexpr int DZ = WS_HY * WS_HX, DY = WS_HX;
    bool tile_changed = false;
    // voxel-by-voxel (Gauss-Seidel) sweeps: each voxel against its six neighbours
    for (;;) {
        bool chg = false;
#pragma unroll
        for (int k = 0; k < WS_VPT; ++k) {
            const int j = tid + k * WS_T;
            const int vz = j / (WS_Y * WS_X), vy = (j / WS_X) % WS_Y, vx = j % WS_X;
            if (vz >= lz || vy >= ly || vx >= lx) continue;
            const int h = ((vz + 1) * WS_HY + vy + 1) * WS_HX + vx + 1;
            const u32 c = C[h];
            if (c == 0u) continue;                               // a seed
            const u32 f = F[j];
            const u32 nb[6] = {C[h - DZ], C[h + DZ], C[h - DY], C[h + DY], C[h - 1], C[h + 1]};
            if (PHASE == 1) {
                u32 best = min(min(min(nb[0], nb[1]), min(nb[2], nb[3])), min(nb[4], nb[5]));
                const u32 cand = best == WS_INF ? WS_INF : max(best, f);
                if (cand < c) { C[h] = cand; chg = true; }
            } else {
                if (c == WS_INF) continue;
                const int off[6] = {-DZ, DZ, -DY, DY, -1, 1};
                u32 l = Lsh[h];
                const u32 l0 = l;
#pragma unroll
                for (int d = 0; d < 6; ++d)
                    if (nb[d] != WS_INF && max(nb[d], f) == c) l = min(l, Lsh[h + off[d]]);
                if (l < l0) { Lsh[h] = l; chg = true; }
            }
        }
        if (!__syncthreads_or(chg)) break;
        tile_changed = true;
    }
    if (!tile_changed) return;
    for (int j = tid; j < WS_Z * WS_Y * WS_X; j += WS_T) {
        const int vz = j / (WS_Y * WS_X), vy = (j / WS_X) % WS_Y, vx = j % WS_X;
        if (vz >= lz || vy >= ly || vx >= lx) continue;
        const int h = ((vz + 1) * WS_HY + vy + 1) * WS_HX + vx + 1;
        const int64_t o = (int64_t)(z0 + vz) * YX + (int64_t)(y0 + vy) * g.S[2] + (x0 + vx);
        if (PHASE == 1) cost[o] = C[h]; else lab[o] = Lsh[h];
    }
    if (tid < 6) {
        // the six neighbour tiles of the same block see a new halo: each goes on the next round's
        // list once (stamp = the round that listed it)
        const int64_t zs = (int64_t)n1 * n2;
        bool ok = false;
        int64_t u = 0;
        switch (tid) {
            case 0: ok = iz > 0 && g.tblk[0][iz - 1] == bz; u = t - zs; break;
            case 1: ok = iz + 1 < g.nt[0] && g.tblk[0][iz + 1] == bz; u = t + zs; break;
            case 2: ok = iy > 0 && g.tblk[1][iy - 1] == by; u = t - n2; break;
            case 3: ok = iy + 1 < g.nt[1] && g.tblk[1][iy + 1] == by; u = t + n2; break;
            case 4: ok = ix > 0 && g.tblk[2][ix - 1] == bx; u = t - 1; break;
            default: ok = ix + 1 < g.nt[2] && g.tblk[2][ix + 1] == bx; u = t + 1; break;
        }
        if (ok && atomicExch(&stamp[u], round) != round) list_out[atomicAdd(n_out, 1u)] = (u32)u;
    }
}

__global__ void k_ws_write(int64_t n, const u32* __restrict__ lab, const u8* __restrict__ mask, u64* out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const u32 l = lab[i];
        out[i] = (l == WS_INF || (mask && !mask[i])) ? 0ull : (u64)l;
    }
}

}  // namespace cc

extern "C" int cc_watershed_from_seeds(cc_ctx* c, const float* in, const uint64_t* seeds, const uint8_t* mask,
                                       const int64_t shape[3], const int64_t block_shape[3], uint64_t* out,
                                       int64_t* rounds) {
    CC_TRY({
        CC_REQUIRE(c && in && seeds && out && shape && block_shape, "NULL argument");
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
        HIP_OK(hipMemsetAsync(smin, 0xFF, nb * sizeof(u32), s));
        HIP_OK(hipMemsetAsync(smax, 0x00, 2 * nb * sizeof(u32), s));
        launch(c, "k_block_stats", [&] { k_block_stats<<<(unsigned)gg.n_tiles, NTHREADS, 0, s>>>(gg, in, smin, smax, sflag); });
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
        c->ws_buf.ensure((size_t)n * 2 * sizeof(u32) + 3 * (size_t)nt * sizeof(u32) + 64);
        u32* cost = c->ws_buf.as<u32>();
        u32* lab = cost + n;
        u32* stamp = lab + n;
        u32* list0 = stamp + nt;
        u32* list1 = list0 + nt;
        c->counter.ensure(4 * sizeof(u32));
        u32* flags = c->counter.as<u32>();            // [0] seed id overflow, [1] tiles listed for the next round
        HIP_OK(hipMemsetAsync(flags, 0, 4 * sizeof(u32), s));
        HIP_OK(hipMemsetAsync(stamp, 0, nt * sizeof(u32), s));
        launch(c, "k_ws_init", [&] { k_ws_init<<<grid_stride(n), 256, 0, s>>>(n, seeds, cost, lab, flags); });
        int64_t total_rounds = 0;
        u32 round = 0;
        for (int phase = 1; phase <= 2; ++phase) {
            // the first round of a phase visits every tile, later rounds the tiles listed by the last
            const u32* lin = nullptr;
            int64_t ntile = nt;
            for (int64_t r = 0; ntile > 0; ++r) {
                CC_REQUIRE(r < 4 * n + 16, "watershed did not converge");
                ++round;
                HIP_OK(hipMemsetAsync(flags + 1, 0, sizeof(u32), s));
                launch(c, phase == 1 ? "k_ws_relax_cost" : "k_ws_relax_label", [&] {
                    if (phase == 1)
                        k_ws_relax<1><<<(unsigned)ntile, WS_T, 0, s>>>(g, in, mask, smin, smax, sflag, cost, lab, lin, stamp,
                                                                      round, list1, flags + 1);
                    else
                        k_ws_relax<2><<<(unsigned)ntile, WS_T, 0, s>>>(g, in, mask, smin, smax, sflag, cost, lab, lin, stamp,
                                                                      round, list1, flags + 1);
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
                ntile = fl[1];
            }
        }
        launch(c, "k_ws_write", [&] { k_ws_write<<<grid_stride(n), 256, 0, s>>>(n, lab, mask, out); });
        sync(c);
        if (rounds) *rounds = total_rounds;
    })
}
