// cc_relabel.hip -- consecutive relabelling on the MI355X (included at the end of cc_lib.hip,
// after cc_eval.hip whose hash helpers it shares).
//
// Replaces the reference RelabelWorkflow (relabel/relabel_workflow.py:10-60): FindUniques
// (find_uniques.py, np.unique per block), FindLabeling (find_labeling.py:84-120: sorted uniques,
// new ids consecutive from 0 when 0 occurs, else from 1; the (old, new) assignment table) and
// Write (write.py, apply the table).  Device: one pass inserts every x-run of equal ids into an
// HBM open-addressing set (run heads by one ballot per 64 voxels; a hit on an existing key is a
// plain load, no atomic), the set is compacted and radix-sorted, every sorted id's slot receives
// its new id, and one more pass maps the volume (16 B/voxel: 8 read + 8 write).

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

constexpr int RL_Q = 4;     // 64-voxel groups per wave iteration (loads in flight)

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

// Each workgroup owns a contiguous voxel range and an LDS set: only ids new to the workgroup
// reach the HBM set.  (Global inserts per x-run measured 6.4-7 s at C3: ~67 M waves probing the
// background id's slot, with agent-scope loads or with CAS on stale L2 lines alike.)
__global__ __launch_bounds__(256) void k_rl_unique(const u64* __restrict__ lab, int64_t n, int64_t per_wg, u64* keys,
                                                   u64 mask, u32* err) {
    __shared__ u64 lk[EV_LDS];
    for (int e = threadIdx.x; e < EV_LDS; e += 256) lk[e] = EV_EMPTY;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int64_t beg = (int64_t)blockIdx.x * per_wg, end = min(n, beg + per_wg);
    u32 e_or = 0;
    for (int64_t base = beg + (threadIdx.x & ~63) * RL_Q; base < end; base += 256 * RL_Q) {
        u64 v[RL_Q];
#pragma unroll
        for (int q = 0; q < RL_Q; ++q) {
            const int64_t i = base + q * 64 + lane;
            v[q] = i < end ? __builtin_nontemporal_load(lab + i) : EV_EMPTY;
            if (i < end && v[q] == EV_EMPTY) e_or |= EV_ERR_GT;
        }
#pragma unroll
        for (int q = 0; q < RL_Q; ++q) {
            const u64 prev = (u64)__shfl_up((unsigned long long)v[q], 1);
            if ((lane == 0 || v[q] != prev) && v[q] != EV_EMPTY) {
                const u64 key = v[q];
                u32 h = (u32)ev_hash(key) & (EV_LDS - 1);
                int probe = 0;
                for (; probe < EV_LDS_PROBES; ++probe) {
                    u64 k = lk[h];
                    if (k == EV_EMPTY) {
                        k = atomicCAS((unsigned long long*)&lk[h], (unsigned long long)EV_EMPTY, (unsigned long long)key);
                        if (k == EV_EMPTY) {                  // new to this workgroup
                            if (!rl_insert(keys, mask, key)) e_or |= EV_ERR_FULL;
                            break;
                        }
                    }
                    if (k == key) break;
                    h = (h + 1) & (EV_LDS - 1);
                }
                if (probe == EV_LDS_PROBES && !rl_insert(keys, mask, key)) e_or |= EV_ERR_FULL;
            }
        }
    }
    if (e_or) atomicOr(err, e_or);
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

// out[i] = new id of lab[i]; run heads look the id up, the rest of the run takes the head's value
__global__ __launch_bounds__(256) void k_rl_apply(const u64* lab, int64_t n, const u64* __restrict__ keys, u64 mask,
                                                  const u64* __restrict__ vals, u64* out) {
    const int lane = threadIdx.x & 63;
    const int64_t stride = (int64_t)gridDim.x * 256 * RL_Q;
    for (int64_t base = (int64_t)blockIdx.x * 256 * RL_Q + (threadIdx.x & ~63) * RL_Q; base < n; base += stride) {
        u64 v[RL_Q];
#pragma unroll
        for (int q = 0; q < RL_Q; ++q) {
            const int64_t i = base + q * 64 + lane;
            v[q] = i < n ? __builtin_nontemporal_load(lab + i) : EV_EMPTY;
        }
#pragma unroll
        for (int q = 0; q < RL_Q; ++q) {
            const int64_t i = base + q * 64 + lane;
            const u64 prev = (u64)__shfl_up((unsigned long long)v[q], 1);
            const bool head = lane == 0 || v[q] != prev;
            const u64 H = __ballot(head);
            u64 nv = 0;
            if (head && v[q] != EV_EMPTY) nv = vals[rl_slot(keys, mask, v[q])];
            const int hl = 63 - __builtin_clzll(H & (lane == 63 ? ~0ull : ((2ull << lane) - 1)));
            nv = (u64)__shfl((unsigned long long)nv, hl);
            if (i < n) __builtin_nontemporal_store(nv, out + i);
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
        hipStream_t s = c->stream;
        *n_unique = 0;
        *start_label = 1;
        if (n == 0) return 0;
        const unsigned grid = std::min<unsigned>(4096, grid_stride((n + RL_Q - 1) / RL_Q));
        // k_rl_unique: contiguous ranges of whole 256 * RL_Q steps, ~8192 workgroups
        const int64_t step = 256 * RL_Q, steps = (n + step - 1) / step;
        const int64_t per_wg = ((steps + 8191) / 8192) * step;
        const unsigned ugrid = (unsigned)((n + per_wg - 1) / per_wg);
        c->counter.ensure(2 * sizeof(u32));
        int64_t cap = std::max<int64_t>(c->rl_cap, 1 << 16);   // grown tables are kept for the next call
        for (;;) {
            c->ev_seg.ensure(2 * cap * sizeof(u64));     // keys | new ids
            u64* keys = c->ev_seg.as<u64>();
            u64* vals = keys + cap;
            HIP_OK(hipMemsetAsync(keys, 0xFF, cap * sizeof(u64), s));
            HIP_OK(hipMemsetAsync(c->counter.p, 0, 2 * sizeof(u32), s));
            u32* err = c->counter.as<u32>();
            launch(c, "k_rl_unique", [&] { k_rl_unique<<<ugrid, 256, 0, s>>>(labels, n, per_wg, keys, (u64)cap - 1, err); });
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
            size_t tmp = 0;
            HIP_OK(hipcub::DeviceRadixSort::SortKeys(nullptr, tmp, comp, sorted, (int)nu, 0, 64, s));
            c->cub_tmp.ensure(tmp);
            launch(c, "radix_sort", [&] {
                HIP_OK(hipcub::DeviceRadixSort::SortKeys(c->cub_tmp.p, tmp, comp, sorted, (int)nu, 0, 64, s));
            });
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
            launch(c, "k_rl_apply", [&] { k_rl_apply<<<grid, 256, 0, s>>>(labels, n, keys, (u64)cap - 1, vals, out); });
            if (uniques_host && cap_host > 0)
                HIP_OK(hipMemcpyAsync(uniques_host, sorted, std::min<int64_t>(cap_host, nu) * sizeof(u64),
                                      hipMemcpyDeviceToHost, s));
            sync(c);
            return 0;
        }
    })
}

}  // extern "C"
