// cc_eval.hip -- segmentation evaluation on the MI355X (included at the end of cc_lib.hip).
//
// Replaces the reference EvaluationWorkflow (evaluation/evaluation_workflow.py:46-84):
//   1. NodeLabelWorkflow overlaps (node_labels/block_node_labels.py:133-166): per block of the
//      evaluation block grid, skipped when the segmentation block sums to 0 (:141-145); voxels
//      whose ground-truth label equals ignore_label are not counted (withIgnoreLabel, :159-162);
//      overlaps[seg id][gt id] = voxel count.
//   2. measures (evaluation/measures.py:81-162): the contingency table over all blocks, sizes of
//      the gt ids (a) and seg ids (b), n_points, then VI split / merge (log2) and the adapted rand
//      error / rand index.
//
// Device layout: one pass over (seg, gt) uint64 volumes, 16 B/voxel, HBM-bound.  A wave takes
// 512 voxels of one x-row as 8 coalesced loads of 64 voxels; runs of equal (seg, gt) keys among
// the 64 lanes are found with one ballot and only each run's head lane touches a table.  Each
// workgroup owns consecutive rows and a 2048-entry LDS hash table, flushed once to the global
// open-addressing tables at the end.  Pairs of a seg-0 voxel are kept apart per block
// (ZTAG keys: block id, gt id) because whether they count depends on the whole block (the
// ws.sum() == 0 skip); k_ev_fold adds them for blocks that held any non-zero seg voxel.
// Then k_ev_sizes builds the per-id size tables from the pair table and k_ev_reduce produces
// per-workgroup partial sums (sum c, sum c^2, sum c log2 c, entries) of each table, summed on
// the host in a fixed order.
//
// Key packing (64 bit): pair key = seg << 32 | gt (seg < 2^31, gt < 2^32 - 1);
// seg-0 key = ZTAG | block << 32 | gt; EMPTY = all ones.  Ids outside these ranges fail loudly.

namespace cc {

constexpr u64 EV_EMPTY = ~0ull;
constexpr u64 EV_ZTAG = 1ull << 63;
constexpr int EV_LDS = 2048;       // LDS hash entries per workgroup
constexpr int EV_LDS_PROBES = 32;
constexpr int EV_PROBES = 1024;    // global probe limit before reporting the table as full (a full
                                   // table costs every further insert this many probes before the rerun)
constexpr int EV_Q = 8;            // loads of 64 voxels per wave item
constexpr int EV_ROW = 64 * EV_Q;  // voxels of one row per wave item
constexpr u32 EV_ERR_SEG = 1, EV_ERR_GT = 2, EV_ERR_FULL = 4;

__device__ __forceinline__ u64 ev_hash(u64 k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}

// global open-addressing insert (linear probing); false when EV_PROBES slots were taken
__device__ bool ev_insert(u64* keys, u64* cnts, u64 mask, u64 key, u64 c) {
    u64 h = ev_hash(key) & mask;
    for (int probe = 0; probe < EV_PROBES; ++probe) {
        u64 k = __hip_atomic_load(&keys[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (k == EV_EMPTY) {
            k = atomicCAS((unsigned long long*)&keys[h], (unsigned long long)EV_EMPTY, (unsigned long long)key);
            if (k == EV_EMPTY) k = key;
        }
        if (k == key) {
            atomicAdd((unsigned long long*)&cnts[h], (unsigned long long)c);
            return true;
        }
        h = (h + 1) & mask;
    }
    return false;
}

struct EvTabs {
    u64 *mk, *mc;   // pairs (seg << 32 | gt)
    u64 *zk, *zc;   // seg-0 pairs per block
    u64 mask;       // capacity - 1 (power of two)
    u32* err;
};

__device__ __forceinline__ void ev_global(const EvTabs& t, u64 key, u64 c) {
    const bool ok = (key & EV_ZTAG) ? ev_insert(t.zk, t.zc, t.mask, key, c) : ev_insert(t.mk, t.mc, t.mask, key, c);
    if (!ok) atomicOr(t.err, EV_ERR_FULL);
}

__device__ __forceinline__ void ev_local(u64* lk, u32* lc, const EvTabs& t, u64 key, u32 c) {
    u32 h = (u32)ev_hash(key) & (EV_LDS - 1);
    for (int probe = 0; probe < EV_LDS_PROBES; ++probe) {
        u64 k = lk[h];
        if (k == EV_EMPTY) {
            k = atomicCAS((unsigned long long*)&lk[h], (unsigned long long)EV_EMPTY, (unsigned long long)key);
            if (k == EV_EMPTY) k = key;
        }
        if (k == key) {
            atomicAdd(&lc[h], c);
            return;
        }
        h = (h + 1) & (EV_LDS - 1);
    }
    ev_global(t, key, c);   // LDS table crowded: straight to HBM
}

// blocks of the evaluation grid, walked incrementally along x
struct EvGrid {
    int64_t Y, X, bz, by, bx, nby, nbx;
};

// One wave item = 512 voxels of one x-row (8 loads of 64 consecutive uint64 per volume, each
// instruction one contiguous 512-B span).  After each load, runs of equal keys across the 64
// lanes are found with one ballot (run heads) and only the head lane of each run adds
// (key, run length) to the LDS table.  A workgroup owns `rows_per_wg` consecutive rows.
__global__ __launch_bounds__(256) void k_ev_overlaps(const u64* __restrict__ seg, const u64* __restrict__ gt,
                                                     int64_t n_rows, int64_t rows_per_wg, EvGrid gr, int use_ignore,
                                                     u64 ignore, EvTabs t, u32* __restrict__ blk_flag) {
    __shared__ u64 lk[EV_LDS];
    __shared__ u32 lc[EV_LDS];
    for (int e = threadIdx.x; e < EV_LDS; e += 256) { lk[e] = EV_EMPTY; lc[e] = 0; }
    __syncthreads();
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_wg, r1 = min(n_rows, r0 + rows_per_wg);
    const int64_t nseg = (gr.X + EV_ROW - 1) / EV_ROW;
    const int64_t items = (r1 - r0) * nseg;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    u32 err = 0, flagged = NONE;
    for (int64_t it = wave; it < items; it += 4) {
        const int64_t ri = it / nseg;
        const int64_t row = r0 + ri;
        const int64_t x0 = (it - ri * nseg) * EV_ROW;
        const int64_t z = row / gr.Y, y = row - z * gr.Y;
        const u64 rowbid = (u64)(((z / gr.bz) * gr.nby + y / gr.by) * gr.nbx);
        const u64* sp = seg + row * gr.X;
        const u64* gp = gt + row * gr.X;
        u64 sv[EV_Q], gv[EV_Q];
#pragma unroll
        for (int q = 0; q < EV_Q; ++q) {
            const int64_t x = x0 + q * 64 + lane;
            sv[q] = x < gr.X ? __builtin_nontemporal_load(sp + x) : 0;
            gv[q] = x < gr.X ? __builtin_nontemporal_load(gp + x) : 0;
        }
        int64_t xb = (x0 + lane) / gr.bx, xr = (x0 + lane) - xb * gr.bx;
#pragma unroll
        for (int q = 0; q < EV_Q; ++q) {
            const bool valid = x0 + q * 64 + lane < gr.X;
            const u64 s = sv[q], g = gv[q];
            const u64 bid = rowbid + (u64)xb;
            // block_node_labels.py:141: the block counts when its seg is not all 0, whatever the gt
            if (valid && s != 0 && (u32)bid != flagged) {
                if (blk_flag[bid] == 0) blk_flag[bid] = 1;
                flagged = (u32)bid;
            }
            u64 key = EV_EMPTY;
            if (valid && !(use_ignore && g == ignore)) {
                // ids beyond the packing make no key (a seg id >= 2^31 would carry EV_ZTAG and a
                // garbage block index into k_ev_fold): the call reports them and the caller
                // relabels (Context.evaluate)
                if (s >> 31) err |= EV_ERR_SEG;
                if (g >= 0xFFFFFFFFull) err |= EV_ERR_GT;
                if (!(s >> 31) && g < 0xFFFFFFFFull) key = s == 0 ? (EV_ZTAG | (bid << 32) | g) : ((s << 32) | g);
            }
            const u64 prev = (u64)__shfl_up((unsigned long long)key, 1);
            const bool head = lane == 0 || key != prev;
            const u64 H = __ballot(head);
            if (head && key != EV_EMPTY) {
                const u64 above = lane == 63 ? 0 : H >> (lane + 1);
                const u32 len = above ? (u32)__builtin_ctzll(above) + 1 : (u32)(64 - lane);
                ev_local(lk, lc, t, key, len);
            }
            xr += 64;
            while (xr >= gr.bx) { xr -= gr.bx; ++xb; }
        }
    }
    if (err) atomicOr(t.err, err);
    __syncthreads();
    for (int e = threadIdx.x; e < EV_LDS; e += 256)
        if (lk[e] != EV_EMPTY) ev_global(t, lk[e], lc[e]);
}

// seg-0 pairs of the blocks that held any non-zero seg voxel join the pair table as (0, gt)
__global__ __launch_bounds__(256) void k_ev_fold(EvTabs t, const u32* __restrict__ blk_flag) {
    const u64 cap = t.mask + 1;
    for (u64 e = (u64)blockIdx.x * 256 + threadIdx.x; e < cap; e += (u64)gridDim.x * 256) {
        const u64 k = t.zk[e];
        if (k == EV_EMPTY) continue;
        const u32 bid = (u32)((k >> 32) & 0x7FFFFFFFu);
        if (blk_flag[bid]) ev_global(t, k & 0xFFFFFFFFull, t.zc[e]);
    }
}

// size tables: seg id -> sum of its pair counts (b_dict), gt id -> (a_dict); measures.py:81-89
__global__ __launch_bounds__(256) void k_ev_sizes(EvTabs t, u64* sk, u64* sc, u64* gk, u64* gc) {
    const u64 cap = t.mask + 1;
    bool ok = true;
    // wave-uniform trip count: the ballot below needs every lane
    for (u64 e0 = (u64)blockIdx.x * 256 + (threadIdx.x & ~63u); e0 < cap; e0 += (u64)gridDim.x * 256) {
        const u64 e = e0 + (threadIdx.x & 63);
        const u64 k = e < cap ? t.mk[e] : EV_EMPTY;
        const u64 c = k != EV_EMPTY ? t.mc[e] : 0;
        const u64 sid = k != EV_EMPTY ? k >> 32 : EV_EMPTY;
        if (k != EV_EMPTY) ok = ev_insert(gk, gc, t.mask, k & 0xFFFFFFFFull, c) && ok;
        // seg ids repeat across many pairs (seg 0 against every gt object): one add per wave
        // when every occupied slot of the wave holds the same seg id
        const int first = __builtin_ctzll(__ballot(k != EV_EMPTY) | (1ull << 63));
        const u64 s0 = (u64)__shfl((unsigned long long)sid, first);
        if (__all(k == EV_EMPTY || sid == s0)) {
            u64 sum = c;
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) sum += (u64)__shfl_xor((unsigned long long)sum, o);
            if ((int)(threadIdx.x & 63) == first && k != EV_EMPTY) ok = ev_insert(sk, sc, t.mask, s0, sum) && ok;
        } else if (k != EV_EMPTY) {
            ok = ev_insert(sk, sc, t.mask, sid, c) && ok;
        }
    }
    if (!ok) atomicOr(t.err, EV_ERR_FULL);
}

// per-workgroup partials of one table: {entries, sum c} (u64) and {sum c^2, sum c log2 c} (f64)
__global__ __launch_bounds__(256) void k_ev_reduce(const u64* __restrict__ keys, const u64* __restrict__ cnts, u64 cap,
                                                   u64* __restrict__ pu, double* __restrict__ pf) {
    u64 ne = 0, sc = 0;
    double s2 = 0, sl = 0;
    for (u64 e = (u64)blockIdx.x * 256 + threadIdx.x; e < cap; e += (u64)gridDim.x * 256) {
        if (keys[e] == EV_EMPTY) continue;
        const u64 c = cnts[e];
        const double d = (double)c;
        ne += 1;
        sc += c;
        s2 += d * d;
        sl += d * log2(d);
    }
    __shared__ u64 su[2][4];
    __shared__ double sf[2][4];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        ne += (u64)__shfl_xor((unsigned long long)ne, o);
        sc += (u64)__shfl_xor((unsigned long long)sc, o);
        s2 += __shfl_xor(s2, o);
        sl += __shfl_xor(sl, o);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { su[0][w] = ne; su[1][w] = sc; sf[0][w] = s2; sf[1][w] = sl; }
    __syncthreads();
    if (threadIdx.x == 0) {
        pu[2 * blockIdx.x] = su[0][0] + su[0][1] + su[0][2] + su[0][3];
        pu[2 * blockIdx.x + 1] = su[1][0] + su[1][1] + su[1][2] + su[1][3];
        pf[2 * blockIdx.x] = ((sf[0][0] + sf[0][1]) + sf[0][2]) + sf[0][3];
        pf[2 * blockIdx.x + 1] = ((sf[1][0] + sf[1][1]) + sf[1][2]) + sf[1][3];
    }
}

}  // namespace cc

static constexpr int EV_REDUCE_WG = 512;

struct EvSums {
    uint64_t entries = 0, sum = 0;
    double sq = 0, clog = 0;
};

static EvSums ev_table_sums(cc_ctx* c, const u64* keys, const u64* cnts, int64_t cap, u64* pu, double* pf) {
    hipStream_t s = cstream(c);
    launch(c, "k_ev_reduce", [&] { k_ev_reduce<<<EV_REDUCE_WG, 256, 0, s>>>(keys, cnts, (u64)cap, pu, pf); });
    std::vector<u64> hu(2 * EV_REDUCE_WG);
    std::vector<double> hf(2 * EV_REDUCE_WG);
    HIP_OK(hipMemcpyAsync(hu.data(), pu, hu.size() * sizeof(u64), hipMemcpyDeviceToHost, s));
    HIP_OK(hipMemcpyAsync(hf.data(), pf, hf.size() * sizeof(double), hipMemcpyDeviceToHost, s));
    sync(c);
    EvSums r;
    for (int i = 0; i < EV_REDUCE_WG; ++i) {
        r.entries += hu[2 * i];
        r.sum += hu[2 * i + 1];
        r.sq += hf[2 * i];
        r.clog += hf[2 * i + 1];
    }
    return r;
}

// ids beyond the 64-bit key packing: reported with their own status (CC_ERR_ID_RANGE) so a caller
// can relabel and retry without parsing the message
struct CCIdRangeError : CCError {};

static int evaluate_impl(cc_ctx* c, const uint64_t* seg, const uint64_t* gt, const int64_t shape[3],
                         const int64_t block_shape[3], int use_ignore, uint64_t ignore_label, cc_eval_result* out);

extern "C" {

int cc_evaluate(cc_ctx* c, const uint64_t* seg, const uint64_t* gt, const int64_t shape[3],
                const int64_t block_shape[3], int use_ignore, uint64_t ignore_label, cc_eval_result* out) {
    try {
        return evaluate_impl(c, seg, gt, shape, block_shape, use_ignore, ignore_label, out);
    } catch (const CCIdRangeError& e) {
        g_err = e.msg;
        return CC_ERR_ID_RANGE;
    } catch (const CCError& e) {
        g_err = e.msg;
        return -1;
    } catch (const std::exception& e) {
        g_err = e.what();
        return -2;
    }
}

}  // extern "C"

static int evaluate_impl(cc_ctx* c, const uint64_t* seg, const uint64_t* gt, const int64_t shape[3],
                         const int64_t block_shape[3], int use_ignore, uint64_t ignore_label, cc_eval_result* out) {
    {
        CC_REQUIRE(c && seg && gt && shape && block_shape && out, "bad arguments");
        HIP_OK(hipSetDevice(c->device));
        hipStream_t s = cstream(c);
        int64_t nb[3];
        for (int a = 0; a < 3; ++a) {
            CC_REQUIRE(shape[a] >= 1 && block_shape[a] >= 1, "shape and block_shape must be >= 1");
            nb[a] = (shape[a] + block_shape[a] - 1) / block_shape[a];
        }
        const int64_t n_blocks = nb[0] * nb[1] * nb[2];
        CC_REQUIRE(n_blocks < (1LL << 31), "too many evaluation blocks (>= 2^31)");
        CC_REQUIRE(((uintptr_t)seg & 7) == 0 && ((uintptr_t)gt & 7) == 0, "seg / gt must be 8-byte aligned");
        EvGrid gr{shape[1], shape[2], block_shape[0], block_shape[1], block_shape[2], nb[1], nb[2]};
        // rows of one workgroup: ~8192 workgroups on large volumes (LDS tables stay sparse)
        const int64_t n_rows = shape[0] * shape[1];
        const int64_t rows_per_wg = std::max<int64_t>(1, (n_rows + 8191) / 8192);
        const int64_t n_wg = (n_rows + rows_per_wg - 1) / rows_per_wg;
        CC_REQUIRE(n_wg < (1LL << 31), "too many rows");
        const unsigned grid = (unsigned)n_wg;
        c->ev_flag.ensure(n_blocks * sizeof(u32) + 16);
        c->ev_part.ensure(4 * EV_REDUCE_WG * sizeof(u64));
        c->counter.ensure(sizeof(u32));
        // 2^20 slots (16 MB per table) to start: C3-sized partitions hold ~150 k pairs, and a table
        // that fills up costs a slow pass plus a rerun (the 80 ms first call of round 2)
        int64_t cap = std::max<int64_t>(c->ev_cap, 1 << 20);
        for (;;) {
            c->ev_main.ensure(2 * cap * sizeof(u64));
            c->ev_z.ensure(2 * cap * sizeof(u64));
            c->ev_seg.ensure(2 * cap * sizeof(u64));
            c->ev_gt.ensure(2 * cap * sizeof(u64));
            u64* mk = c->ev_main.as<u64>();
            u64* zk = c->ev_z.as<u64>();
            u64* sk = c->ev_seg.as<u64>();
            u64* gk = c->ev_gt.as<u64>();
            for (u64* k : {mk, zk, sk, gk}) {
                HIP_OK(hipMemsetAsync(k, 0xFF, cap * sizeof(u64), s));
                HIP_OK(hipMemsetAsync(k + cap, 0, cap * sizeof(u64), s));
            }
            HIP_OK(hipMemsetAsync(c->ev_flag.p, 0, n_blocks * sizeof(u32), s));
            HIP_OK(hipMemsetAsync(c->counter.p, 0, sizeof(u32), s));
            EvTabs t{mk, mk + cap, zk, zk + cap, (u64)cap - 1, c->counter.as<u32>()};
            u32* flag = c->ev_flag.as<u32>();
            launch(c, "k_ev_overlaps", [&] {
                k_ev_overlaps<<<grid, 256, 0, s>>>(seg, gt, n_rows, rows_per_wg, gr, use_ignore ? 1 : 0, ignore_label, t, flag);
            });
            launch(c, "k_ev_fold", [&] { k_ev_fold<<<grid_stride(cap), 256, 0, s>>>(t, flag); });
            launch(c, "k_ev_sizes", [&] { k_ev_sizes<<<std::min<unsigned>(2048, grid_stride(cap)), 256, 0, s>>>(t, sk, sk + cap, gk, gk + cap); });
            u32 herr = 0;
            HIP_OK(hipMemcpyAsync(&herr, c->counter.p, sizeof(u32), hipMemcpyDeviceToHost, s));
            sync(c);
            if (herr & EV_ERR_SEG) throw CCIdRangeError{{"segmentation id >= 2^31 (evaluation keys pack seg ids in 31 bits)"}};
            if (herr & EV_ERR_GT) throw CCIdRangeError{{"ground-truth id >= 2^32 - 1 (evaluation keys pack gt ids in 32 bits)"}};
            u64* pu = c->ev_part.as<u64>();
            double* pf = (double*)(pu + 2 * EV_REDUCE_WG);
            EvSums m{};
            if (!(herr & EV_ERR_FULL)) m = ev_table_sums(c, mk, mk + cap, cap, pu, pf);
            // keep every table at most half full (linear probing); grow and rerun otherwise
            if ((herr & EV_ERR_FULL) || (int64_t)m.entries * 2 > cap) {
                CC_REQUIRE(cap < (1LL << 31), "contingency table larger than 2^30 pairs");
                cap *= 4;
                continue;
            }
            const EvSums a = ev_table_sums(c, gk, gk + cap, cap, pu, pf);   // gt sizes (a_dict)
            const EvSums b = ev_table_sums(c, sk, sk + cap, cap, pu, pf);   // seg sizes (b_dict)
            c->ev_cap = cap;
            std::memset(out, 0, sizeof(*out));
            out->n_points = m.sum;
            out->n_pairs = m.entries;
            out->n_gt_ids = a.entries;
            out->n_seg_ids = b.entries;
            if (m.sum == 0) return 0;
            CC_REQUIRE(a.sum == m.sum && b.sum == m.sum, "contingency table sizes disagree (measures.py:115)");
            const double np = (double)m.sum, lg = std::log2(np);
            // entropies in bits: H = log2(N) - (1/N) sum c log2 c
            const double h_ab = lg - m.clog / np, h_a = lg - a.clog / np, h_b = lg - b.clog / np;
            out->vi_split = h_ab - h_a;     // H(seg | gt)
            out->vi_merge = h_ab - h_b;     // H(gt | seg)
            const double prec = m.sq / b.sq, rec = m.sq / a.sq;
            out->adapted_rand_error = 1.0 - 2.0 * prec * rec / (prec + rec);
            out->rand_index = 1.0 - (a.sq + b.sq - 2.0 * m.sq) / (np * np);
            out->sum_sq_pairs = m.sq;
            out->sum_sq_gt = a.sq;
            out->sum_sq_seg = b.sq;
            return 0;
        }
    }
}

extern "C" {

int64_t cc_get_overlaps(cc_ctx* c, uint64_t* seg_ids, uint64_t* gt_ids, uint64_t* counts, int64_t cap) {
    try {
        CC_REQUIRE(c, "ctx is NULL");
        CC_REQUIRE(c->ev_cap > 0, "no evaluation has run on this ctx");
        HIP_OK(hipSetDevice(c->device));
        const int64_t tc = c->ev_cap;
        std::vector<u64> h(2 * tc);
        HIP_OK(hipMemcpyAsync(h.data(), c->ev_main.p, 2 * tc * sizeof(u64), hipMemcpyDeviceToHost, cstream(c)));
        HIP_OK(hipStreamSynchronize(cstream(c)));
        int64_t k = 0;
        for (int64_t e = 0; e < tc; ++e) {
            if (h[e] == EV_EMPTY) continue;
            if (k < cap && seg_ids && gt_ids && counts) {
                seg_ids[k] = h[e] >> 32;
                gt_ids[k] = h[e] & 0xFFFFFFFFull;
                counts[k] = h[tc + e];
            }
            ++k;
        }
        return k;
    } catch (const CCError& e) {
        g_err = e.msg;
        return -1;
    }
}

}  // extern "C"
