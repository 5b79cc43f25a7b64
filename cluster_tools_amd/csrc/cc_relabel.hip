// cc_relabel.hip -- consecutive relabelling on the MI355X (included at the end of cc_lib.hip,
// after cc_eval.hip whose hash helpers it shares).
//
// Replaces the reference RelabelWorkflow (relabel/relabel_workflow.py:10-60): FindUniques
// (find_uniques.py, np.unique per block), FindLabeling (find_labeling.py:84-120: sorted uniques,
// new ids consecutive from 0 when 0 occurs, else from 1; the (old, new) assignment table) and
// Write (write.py, apply the table).  Device: one pass inserts the head id of every run of equal
// ids into a per-workgroup LDS set and the ids new to the workgroup into an HBM open-addressing
// set (keeping each workgroup's id list), the HBM set is compacted and radix-sorted, every
// sorted id's slot receives its new id, and one more pass maps the volume from per-workgroup
// LDS tables (24 B/voxel over both passes: 8 read, then 8 read + 8 write).

namespace cc {

__device__ __forceinline__ u64 rl_slot(const u64* keys, u64 mask, u64 key) {
    u64 h = ev_hash(key) & mask;
    for (int probe = 0; probe < EV_PROBES; ++probe) {
        const u64 k = keys[h];
        if (k == key || k == EV_EMPTY) return h;
        h = (h + 1) & mask;
    }
    return ~0ull;
}

constexpr int RL_Q = 8;      // loads per lane per wave iteration (RL_Q * VW voxels in flight)
#ifndef CC_RL_QA
#define CC_RL_QA 8
#endif
constexpr int RL_QA = CC_RL_QA;   // the same for k_rl_apply
constexpr int RL_WG = 512;   // threads per workgroup
typedef unsigned long long rl_u64x2 __attribute__((ext_vector_type(2)));
constexpr int RL_LDS_BITS = 11;
static_assert((1 << RL_LDS_BITS) == EV_LDS, "LDS set size");

// slot of an id in a workgroup's LDS set (any hash will do: the set is private to the kernel)
__device__ __forceinline__ u32 rl_lhash(u64 k) {
    return ((u32)k ^ (u32)(k >> 32) * 0x85EBCA6Bu) * 0x9E3779B1u >> (32 - RL_LDS_BITS);
}

// global set insert; false when EV_PROBES slots were taken
__device__ __forceinline__ bool rl_insert(u64* keys, u64 mask, u64 key) {
    u64 h = ev_hash(key) & mask;
    for (int probe = 0; probe < EV_PROBES; ++probe) {
        u64 k = atomicCAS((unsigned long long*)&keys[h], (unsigned long long)EV_EMPTY, (unsigned long long)key);
        if (k == EV_EMPTY || k == key) return true;
        h = (h + 1) & mask;
    }
    return false;
}

// VW consecutive ids per lane (one 8 VW-byte load), run heads: a voxel whose left neighbour
// (in the same lane or the lane below) holds another id; lane 0's first voxel is always a head
template <int VW>
struct RlVec {
    u64 v[VW];
    __device__ __forceinline__ void load(const u64* p, int64_t i, int64_t end) {
        if constexpr (VW == 2) {
            if (i + 1 < end) {
                const rl_u64x2 t = __builtin_nontemporal_load(reinterpret_cast<const rl_u64x2*>(p + i));
                v[0] = t.x; v[1] = t.y;
            } else {
                v[0] = i < end ? p[i] : EV_EMPTY;
                v[1] = EV_EMPTY;
            }
        } else {
            v[0] = i < end ? __builtin_nontemporal_load(p + i) : EV_EMPTY;
        }
    }
};

// run-head mask of a lane's RL_Q x VW ids (bit q VW + j): the id differs from its left neighbour
// (same lane or the lane below; lane 0's first id always), ids 2^64 - 1 past the end excluded;
// e_or |= EV_ERR_GT for a reserved id inside the range
template <int VW, int Q = RL_Q>
__device__ __forceinline__ u32 rl_heads(const RlVec<VW>* x, int64_t base, int64_t end, int lane, u32& e_or) {
    u32 hm = 0;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int64_t i = base + (q * 64 + lane) * VW;
        const u64 prev = (u64)__shfl_up((unsigned long long)x[q].v[VW - 1], 1);
#pragma unroll
        for (int j = 0; j < VW; ++j) {
            const u64 key = x[q].v[j];
            if (i + j < end && key == EV_EMPTY) e_or |= EV_ERR_GT;
            const u64 left = j ? x[q].v[j - 1] : prev;
            if ((key != left || (j == 0 && lane == 0)) && key != EV_EMPTY) hm |= 1u << (q * VW + j);
        }
    }
    return hm;
}

template <int VW, int Q = RL_Q>
__device__ __forceinline__ u64 rl_pick(const RlVec<VW>* x, int b) {
    u64 k = 0;
#pragma unroll
    for (int q = 0; q < Q; ++q)
#pragma unroll
        for (int j = 0; j < VW; ++j) if (q * VW + j == b) k = x[q].v[j];
    return k;
}

// Each workgroup owns a contiguous voxel range and an LDS set: only ids new to the workgroup
// reach the HBM set.  (Global inserts per x-run measured 6.4-7 s at C3: ~67 M waves probing the
// background id's slot, with agent-scope loads or with CAS on stale L2 lines alike.)  The
// workgroup's set is kept as a list (WGL[wg * EV_LDS ..], WGN[wg]; ~0u when the LDS set
// overflowed) so that k_rl_apply can map the same range from LDS alone.
template <int VW>
__global__ __launch_bounds__(RL_WG) void k_rl_unique(const u64* __restrict__ lab, int64_t n, int64_t per_wg,
                                                     u64* keys, u64 mask, u32* err, u64* WGL, u32* WGN) {
    __shared__ u64 lk[EV_LDS];
    __shared__ u32 ln, lovf;
    for (int e = threadIdx.x; e < EV_LDS; e += RL_WG) lk[e] = EV_EMPTY;
    if (threadIdx.x == 0) { ln = 0; lovf = 0; }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int64_t beg = (int64_t)blockIdx.x * per_wg, end = min(n, beg + per_wg);
    u32 e_or = 0, ovf = 0;
    u64 r0 = EV_EMPTY, r1 = EV_EMPTY;                 // this lane's last two head ids (runs alternate)
    auto head = [&](u64 key) {
        if (key == r0 || key == r1) return;
        r1 = r0; r0 = key;
        u32 h = rl_lhash(key);
        int probe = 0;
#pragma unroll 1
        for (; probe < EV_LDS_PROBES; ++probe) {
            u64 k = lk[h];
            if (k == EV_EMPTY) {
                k = atomicCAS((unsigned long long*)&lk[h], (unsigned long long)EV_EMPTY, (unsigned long long)key);
                if (k == EV_EMPTY) {                  // new to this workgroup
                    if (!rl_insert(keys, mask, key)) e_or |= EV_ERR_FULL;
                    return;
                }
            }
            if (k == key) return;
            h = (h + 1) & (EV_LDS - 1);
        }
        ovf = 1;                                      // LDS set crowded: straight to HBM
        if (!rl_insert(keys, mask, key)) e_or |= EV_ERR_FULL;
    };
    for (int64_t base = beg + (int64_t)(threadIdx.x & ~63) * RL_Q * VW; base < end; base += (int64_t)RL_WG * RL_Q * VW) {
        RlVec<VW> x[RL_Q];
#pragma unroll
        for (int q = 0; q < RL_Q; ++q) x[q].load(lab, base + (q * 64 + lane) * VW, end);
        const u32 hm = rl_heads<VW>(x, base, end, lane, e_or);
        // one insert site for all the lane's heads (an inlined copy per voxel spilled SGPRs)
        for (u32 m = hm; m; m &= m - 1) head(rl_pick<VW>(x, __builtin_ctz(m)));
    }
    if (e_or) atomicOr(err, e_or);
    if (ovf) lovf = 1;
    __syncthreads();
    if (lovf) {
        if (threadIdx.x == 0) WGN[blockIdx.x] = ~0u;
        return;
    }
    for (int e = threadIdx.x; e < EV_LDS; e += RL_WG)
        if (lk[e] != EV_EMPTY) WGL[(int64_t)blockIdx.x * EV_LDS + atomicAdd(&ln, 1u)] = lk[e];
    __syncthreads();
    if (threadIdx.x == 0) WGN[blockIdx.x] = ln;
}

__global__ __launch_bounds__(256) void k_rl_compact(const u64* __restrict__ keys, u64 cap, u64* out, u32* count) {
    for (u64 e = (u64)blockIdx.x * 256 + threadIdx.x; e < cap; e += (u64)gridDim.x * 256) {
        const u64 k = keys[e];
        if (k != EV_EMPTY) out[atomicAdd(count, 1u)] = k;
    }
}

// slot of sorted id i receives its new id i + start (find_labeling.py:106-116)
__global__ __launch_bounds__(256) void k_rl_assign(const u64* __restrict__ sorted, int64_t nu, u64 start,
                                                   const u64* __restrict__ keys, u64 mask, u64* vals) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= nu) return;
    vals[rl_slot(keys, mask, sorted[i])] = (u64)i + start;
}

// out[i] = new id of lab[i] over k_rl_unique's workgroup ranges: the workgroup's id list -> LDS
// table (id -> new id), then run heads look their id up in LDS and the rest of a run takes the
// head's value (ballot + shuffle).  A workgroup whose LDS set overflowed looks up in HBM.
template <int VW>
__global__ __launch_bounds__(RL_WG) void k_rl_apply(const u64* lab, int64_t n, int64_t per_wg,
                                                    const u64* __restrict__ keys, u64 mask,
                                                    const u64* __restrict__ vals, const u64* __restrict__ WGL,
                                                    const u32* __restrict__ WGN, u64* out) {
    __shared__ u64 lk[EV_LDS], lv[EV_LDS];
    for (int e = threadIdx.x; e < EV_LDS; e += RL_WG) lk[e] = EV_EMPTY;
    const u32 nl = WGN[blockIdx.x];
    const bool global = nl == ~0u;
    __syncthreads();
    if (!global) {
        for (u32 e = threadIdx.x; e < nl; e += RL_WG) {
            const u64 key = WGL[(int64_t)blockIdx.x * EV_LDS + e];
            const u64 val = vals[rl_slot(keys, mask, key)];
            u32 h = rl_lhash(key);
            while (atomicCAS((unsigned long long*)&lk[h], (unsigned long long)EV_EMPTY, (unsigned long long)key) != EV_EMPTY)
                h = (h + 1) & (EV_LDS - 1);       // the ids are distinct and nl <= EV_LDS
            lv[h] = val;
        }
    }
    __syncthreads();
    u64 mk0 = EV_EMPTY, mv0 = 0, mk1 = EV_EMPTY, mv1 = 0;   // this lane's last two (id, new id)
    auto lookup = [&](u64 key) -> u64 {
        if (key == mk0) return mv0;
        if (key == mk1) return mv1;
        u64 v = 0;
        if (global) {
            v = vals[rl_slot(keys, mask, key)];
        } else {
            u32 h = rl_lhash(key);
            int probe = 0;
            for (; probe < EV_LDS; ++probe) {        // always found: the list holds every id of the range
                if (lk[h] == key) break;
                h = (h + 1) & (EV_LDS - 1);
            }
            v = probe < EV_LDS ? lv[h] : vals[rl_slot(keys, mask, key)];
        }
        mk1 = mk0; mv1 = mv0; mk0 = key; mv0 = v;
        return v;
    };
    const int lane = threadIdx.x & 63;
    const int64_t beg = (int64_t)blockIdx.x * per_wg, end = min(n, beg + per_wg);
    for (int64_t base = beg + (int64_t)(threadIdx.x & ~63) * RL_QA * VW; base < end; base += (int64_t)RL_WG * RL_QA * VW) {
        RlVec<VW> x[RL_QA];
#pragma unroll
        for (int q = 0; q < RL_QA; ++q) x[q].load(lab, base + (q * 64 + lane) * VW, end);
        u32 e_or = 0;
        const u32 hm = rl_heads<VW, RL_QA>(x, base, end, lane, e_or);
#pragma unroll
        for (int q = 0; q < RL_QA; ++q) {
            const int64_t i = base + (q * 64 + lane) * VW;
            const u32 hq = (hm >> (q * VW)) & ((1u << VW) - 1);
            // one lookup site per group of 64 lanes
            u64 nv[VW];
#pragma unroll
            for (int j = 0; j < VW; ++j) nv[j] = 0;
            for (u32 m = hq; m; m &= m - 1) {
                const int b = __builtin_ctz(m);
                u64 key = x[q].v[0];
#pragma unroll
                for (int j = 1; j < VW; ++j) if (j == b) key = x[q].v[j];
                const u64 v = lookup(key);
#pragma unroll
                for (int j = 0; j < VW; ++j) if (j == b) nv[j] = v;
            }
            // voxel 0 of a lane without a head there: the last value of the nearest lane below
            // holding a head (every voxel in between has the same id)
            const u64 H = __ballot(hq != 0);
            const u64 below = lane ? H & ((1ull << lane) - 1) : 0ull;
            const int hl = below ? 63 - __builtin_clzll(below) : 0;
            u64 lastv = 0;
#pragma unroll
            for (int j = 0; j < VW; ++j) if ((hq >> j) & 1u) lastv = nv[j];
            const u64 from = (u64)__shfl((unsigned long long)lastv, hl);
#pragma unroll
            for (int j = 0; j < VW; ++j)
                if (!((hq >> j) & 1u)) nv[j] = j ? nv[j - 1] : from;
            if constexpr (VW == 2) {
                if (i + 1 < end) __builtin_nontemporal_store(rl_u64x2{nv[0], nv[1]}, reinterpret_cast<rl_u64x2*>(out + i));
                else if (i < end) out[i] = nv[0];
            } else {
                if (i < end) __builtin_nontemporal_store(nv[0], out + i);
            }
        }
    }
}

}  // namespace cc

extern "C" {

int cc_relabel_consecutive(cc_ctx* c, const uint64_t* labels, uint64_t* out, int64_t n, uint64_t* n_unique,
                           uint64_t* start_label, uint64_t* uniques_host, int64_t cap_host) {
    CC_TRY({
        CC_REQUIRE(c && labels && out && n >= 0 && n_unique && start_label, "bad arguments");
        HIP_OK(hipSetDevice(c->device));
        hipStream_t s = cstream(c);
        *n_unique = 0;
        *start_label = 1;
        if (n == 0) return 0;
        // both passes: contiguous ranges of whole RL_WG * RL_Q * VW steps, ~8192 workgroups;
        // 16-B accesses when both arrays are 16-B aligned
        const bool vw2 = ((uintptr_t)labels % 16 == 0) && ((uintptr_t)out % 16 == 0);
        const int64_t step = (int64_t)RL_WG * RL_Q * (vw2 ? 2 : 1), steps = (n + step - 1) / step;
        const int64_t per_wg = ((steps + 8191) / 8192) * step;
        const unsigned ugrid = (unsigned)((n + per_wg - 1) / per_wg);
        c->rl_wg.ensure((size_t)ugrid * (EV_LDS * sizeof(u64) + sizeof(u32)));
        u64* WGL = c->rl_wg.as<u64>();
        u32* WGN = reinterpret_cast<u32*>(WGL + (size_t)ugrid * EV_LDS);
        c->counter.ensure(2 * sizeof(u32));
        // id-set slots: at least twice the caller's table capacity (its expected number of distinct
        // ids, bounded by n), so the set is sized right on the first pass -- a set that fills up
        // makes every further insert walk EV_PROBES slots before the pass is rerun larger (the
        // 666 ms first call of round 2); grown sets are kept for the next call
        int64_t cap = std::max<int64_t>(c->rl_cap, 1 << 16);
        if (uniques_host && cap_host > 0) {
            const int64_t want = 2 * std::min<int64_t>(std::min<int64_t>(cap_host, n), 1LL << 27);
            while (cap < want) cap *= 2;
        }
        for (;;) {
            c->ev_seg.ensure(2 * cap * sizeof(u64));     // keys | new ids
            u64* keys = c->ev_seg.as<u64>();
            u64* vals = keys + cap;
            HIP_OK(hipMemsetAsync(keys, 0xFF, cap * sizeof(u64), s));
            HIP_OK(hipMemsetAsync(c->counter.p, 0, 2 * sizeof(u32), s));
            u32* err = c->counter.as<u32>();
            launch(c, "k_rl_unique", [&] {
                if (vw2) k_rl_unique<2><<<ugrid, RL_WG, 0, s>>>(labels, n, per_wg, keys, (u64)cap - 1, err, WGL, WGN);
                else k_rl_unique<1><<<ugrid, RL_WG, 0, s>>>(labels, n, per_wg, keys, (u64)cap - 1, err, WGL, WGN);
            });
            u32 h[2] = {0, 0};
            c->ev_gt.ensure(cap * 2 * sizeof(u64));      // compacted ids | sorted ids
            u64* comp = c->ev_gt.as<u64>();
            u64* sorted = comp + cap;
            launch(c, "k_rl_compact", [&] { k_rl_compact<<<grid_stride(cap), 256, 0, s>>>(keys, (u64)cap, comp, err + 1); });
            HIP_OK(hipMemcpyAsync(h, c->counter.p, 2 * sizeof(u32), hipMemcpyDeviceToHost, s));
            sync(c);
            CC_REQUIRE(!(h[0] & EV_ERR_GT), "label id 2^64 - 1 is reserved");
            if ((h[0] & EV_ERR_FULL) || (int64_t)h[1] * 2 > cap) {
                CC_REQUIRE(cap < (1LL << 31), "more than 2^30 distinct ids");
                cap *= 4;
                continue;
            }
            const int64_t nu = h[1];
            launch(c, "radix_sort", [&] { prims::sort_keys<u64>(comp, sorted, nu, 0, 64, c->cub_tmp, s); });
            u64 first = 1;
            HIP_OK(hipMemcpyAsync(&first, sorted, sizeof(u64), hipMemcpyDeviceToHost, s));
            sync(c);
            const u64 start = first == 0 ? 0 : 1;
            c->rl_cap = cap;
            *n_unique = (uint64_t)nu;
            *start_label = start;
            // the table does not fit the caller's buffer: report its size and leave out_dev
            // untouched (an in-place call must not lose the ids before the table is returned)
            if (uniques_host && cap_host < nu) return 0;
            launch(c, "k_rl_assign", [&] {
                k_rl_assign<<<grid1d(nu), 256, 0, s>>>(sorted, nu, start, keys, (u64)cap - 1, vals);
            });
            launch(c, "k_rl_apply", [&] {
                if (vw2) k_rl_apply<2><<<ugrid, RL_WG, 0, s>>>(labels, n, per_wg, keys, (u64)cap - 1, vals, WGL, WGN, out);
                else k_rl_apply<1><<<ugrid, RL_WG, 0, s>>>(labels, n, per_wg, keys, (u64)cap - 1, vals, WGL, WGN, out);
            });
            if (uniques_host && cap_host > 0)
                HIP_OK(hipMemcpyAsync(uniques_host, sorted, std::min<int64_t>(cap_host, nu) * sizeof(u64),
                                      hipMemcpyDeviceToHost, s));
            sync(c);
            return 0;
        }
    })
}

}  // extern "C"
