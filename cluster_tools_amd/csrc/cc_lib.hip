// cc_lib.hip -- the labelling path: host orchestration and its C ABI (include/cc_mi355x.h).
// First of the library's two translation units (the second, cc_aux.hip, holds evaluation,
// relabelling, prefilter and watershed, so that this unit's code object -- loaded whole at the
// first launch of a one-shot job -- carries only the labelling path's kernels).  Kernels:
// cc_kernels.hip, cc_stage_kernels.hip, cc_generate.hip, cc_mask.hip, and the library's own
// scan / sort / select (cc_prims.hip; no hipcub: see there why).

#include "cc_kernels.hip"
#include "cc_stage_kernels.hip"
#include "cc_generate.hip"
#include "cc_mask.hip"

#include "cc_ctx.hpp"
#include "cc_prims.hip"

// ------------------------------------------------------------------------------------------
// the device pipeline, in phases (single GPU: local -> rid(0) -> final; z-slab shards:
// local -> [allgather of sums] -> rid(base) -> planes -> [seam exchange] -> map -> final)
// ------------------------------------------------------------------------------------------

// stats -> params -> pass1 -> intra-block stitch -> roots -> sort -> offsets (local)
// fast: the one-read-back schedule -- no host read-back in this phase (the k_fix count, the root
// count and the fallback flags stay on the device; see run_pipeline)
static void phase_local(cc_ctx* c, const float* in, const uint8_t* mask, const int64_t shape[3],
                        const int64_t block_shape[3], double threshold, int mode, int64_t zoff,
                        bool local_only, bool fast = false, uint64_t* sum_out = nullptr) {
    require_row_aligned(in, shape[2] * 4);
    require_row_aligned(mask, shape[2]);
    RunState& st = state(c);
    st = RunState();
    st.fast = fast;
    st.hg = make_geom(shape, block_shape, zoff);
    upload_geom(c, st.hg);
    Geom& g = st.hg.g;
    for (int a = 0; a < 3; ++a) st.bs[a] = block_shape[a];
    st.thr = (float)threshold;                // numpy: python float -> float32
    st.mode = mode;
    st.local_only = local_only;
    st.masked = mask != nullptr;
    const int64_t nt = g.n_tiles, nb = g.n_blocks;
    const uint64_t nodes = (uint64_t)nt * g.cap;
    hipStream_t s = cstream(c);

    c->bstat.ensure(nb * 3 * sizeof(u32));
    c->bparam.ensure(2 * nb * sizeof(BlockParam));     // exact parameters, then the guesses (k_sample)
    c->bits.ensure(nt * NROWS * sizeof(u64));
    c->faces.ensure(nt * FACE_STRIDE * sizeof(face_t));
    c->count.ensure(nt * sizeof(u32));
    c->P.ensure(nodes * sizeof(u32));
    c->KR.ensure(nodes * sizeof(u64));
    c->seg.ensure(nb * 2 * sizeof(u32));
    c->values.ensure(nb * sizeof(u64));
    c->offsets.ensure(nb * sizeof(u64));
    c->scalars.ensure(SCALARS * sizeof(u64));

    // block statistics (ordered min, max, NaN flag), accumulated by k_spec
    u32* smin = c->bstat.as<u32>();
    u32* smax = smin + nb;
    u32* sflag = smax + nb;

    BlockParam* bp = c->bparam.as<BlockParam>();
    u64* BITS = c->bits.as<u64>();
    face_t* FACES = c->faces.as<face_t>();
    u32* COUNT = c->count.as<u32>();
    u32* P = c->P.as<u32>();
    u64* KR = c->KR.as<u64>();
    const float thr = st.thr;

    {
        // speculative front: sample -> one read for statistics + pass 1 -> exact parameters ->
        // relabel the tiles whose guessed interval was not exact (see k_spec)
        BlockParam* guess = bp + nb;
        c->spec.ensure((4 * nt + 4 * SAMPLE_PARTS * nb + nt + 1) * sizeof(u32));
        u32* TB = c->spec.as<u32>();
        u32* SPART = TB + 4 * nt;
        u32* FIX = SPART + 4 * SAMPLE_PARTS * nb;
        // seam outputs and flags (big[nb] / iovf[nt]: "any" flags of the global-stitch fallback)
        c->big.ensure(nb + 1);
        c->pairsl.ensure((size_t)nt * TPC * sizeof(u64));
        c->pc.ensure(nt * sizeof(u32));
        c->ipairs.ensure((size_t)nt * TPI * sizeof(u64));
        c->ipc.ensure(nt * sizeof(u32));
        c->iovf.ensure(nt + 1);
        c->rc.ensure((nt + 1) * sizeof(u32));
        c->roff.ensure((nt + 1) * sizeof(u32));
        c->mark.ensure((size_t)(2 * nt + 1) * sizeof(u32) + nt);
        const bool lds_seams = !(c->debug & CC_DEBUG_GLOBAL_STITCH);
        // shards of the one-read-back schedule: the seam pair set and the seam map are cleared here
        const bool shard = fast && sum_out != nullptr;
        if (shard) c->seam_hash.ensure(SEAM_SET * sizeof(u64));
        const int64_t hs_n = shard ? SEAM_SET : 0, hm_n = shard ? (int64_t)c->hm_slots : 0;
        // k_sample's threads first write the front's initial state (FrontClear), then sample
        FrontClear fc;
        {
            fc.nb = nb; fc.nt = nt;
            fc.smin = smin; fc.smax_flag = smax; fc.scalars = c->scalars.as<u64>(); fc.FIX = FIX;
            fc.big = c->big.as<u8>(); fc.iovf = c->iovf.as<u8>(); fc.ipc = c->ipc.as<u32>(); fc.seg = c->seg.as<u32>();
            fc.rc_end = c->rc.as<u32>() + nt; fc.fill = lds_seams ? 0 : 1;
            fc.mflag = fast ? c->mark.as<u32>() : nullptr;
            fc.fchg = fast ? (u8*)(c->mark.as<u32>() + 2 * nt + 1) : nullptr;
            fc.htab = shard ? c->seam_hash.as<u64>() : nullptr; fc.htab_n = hs_n;
            fc.hkeys = hm_n ? c->hmap_keys.as<u64>() : nullptr; fc.hpar = hm_n ? c->hmap_par.as<u32>() : nullptr;
            fc.hm_n = hm_n;
            if (mask) c->mlive.ensure(nb * sizeof(u32));
            fc.mlive = mask ? c->mlive.as<u32>() : nullptr;
            fc.n_clear = std::max<int64_t>({nt + 1, 2 * nb + 1, hs_n, hm_n, (int64_t)SCALARS});   // every scalar, however small the volume
        }
        launch(c, "k_sample", [&] { k_sample<<<(unsigned)(nb * SAMPLE_PARTS), NTHREADS, 0, s>>>(g, in, SPART, fc, mask); });
        launch(c, "k_guess", [&] {
            k_guess<<<(unsigned)((nb + 255) / 256), 256, 0, s>>>(nb, SPART, thr, mode, guess, mask ? c->mlive.as<u32>() : nullptr);
        });
        if (const char* e = std::getenv("CC_SPEC"); e && std::string(e) == "0")     // test hook: no guesses
            HIP_OK(hipMemsetAsync(guess, 0, nb * sizeof(BlockParam), s));
        // masked runs: which blocks hold a mask voxel (the others are skipped, as the reference does)
        const u32* live = mask ? c->mlive.as<u32>() : nullptr;
        if (mask)
            launch(c, "k_mask_live", [&] {
                k_mask_live<<<(unsigned)(nb * LIVE_PARTS), LIVE_THREADS, 0, s>>>(g, mask, c->mlive.as<u32>());
            });
        SpecArgs sa;
        sa.guess = guess;
        sa.smin = smin; sa.smax = smax; sa.sflag = sflag;
        sa.TB = TB;
        sa.live = live;
        auto seams = [&](hipStream_t q, int64_t t0, int64_t t1) {
            launch_on(c, q, "k_seams", [&] {
                k_seams<0><<<(unsigned)((t1 - t0 + SP_WAVES - 1) / SP_WAVES), SP_WAVES * 64, 0, q>>>(
                    g, FACES, COUNT, c->pairsl.as<u64>(), c->pc.as<u32>(), c->big.as<u8>(), c->ipairs.as<u64>(),
                    c->ipc.as<u32>(), c->iovf.as<u8>(), t0, t1, nullptr);
            });
        };
        // The front runs in chunks of whole tile z-layers.  The seams of a chunk read only its
        // faces and those of the layers below, so k_seams of chunk i runs on the side stream
        // while k_spec of chunk i + 1 streams the input (k_seams is latency-bound, k_spec
        // bandwidth-bound).  Tiles k_fix relabels later get their seams recomputed below.
        const int64_t layer = (int64_t)g.nt[1] * g.nt[2];
        const int64_t n_chunks = lds_seams ? std::min<int64_t>(g.nt[0], c->front_chunks) : 1;
        // one chunk (the default): the seams follow on the same stream, no side stream needed
        const hipStream_t ss = n_chunks > 1 ? side_stream(c) : s;
        // the one-read-back schedule with one chunk runs the seams once, after k_fix (whose
        // relabelled tiles then need no second seam pass: k_seams_list and its launch are gone)
        const bool seams_after_fix = fast && n_chunks == 1 && lds_seams;
        if (lds_seams && ss != s) stream_wait(c, s, ss);
        for (int64_t ci = 0; ci < n_chunks; ++ci) {
            const int64_t t0 = g.nt[0] * ci / n_chunks * layer, t1 = g.nt[0] * (ci + 1) / n_chunks * layer;
            sa.t0 = t0;
            const unsigned ng = (unsigned)(t1 - t0);
            launch(c, "k_spec", [&] {
#define CC_SPEC_LAUNCH(M, S) k_spec<M, S><<<ng, NTHREADS, spad, s>>>(g, sa, in, mask, BITS, FACES, COUNT, P, KR)
                const unsigned spad = (unsigned)env_int("CC_LDS_PAD_SPEC", 0);   // A/B only, as CC_LDS_PAD_P2
                if (mask) {
                    if (mode == MODE_GREATER) CC_SPEC_LAUNCH(true, 1);
                    else if (mode == MODE_LESS) CC_SPEC_LAUNCH(true, 2);
                    else CC_SPEC_LAUNCH(true, 3);
                } else {
                    if (mode == MODE_GREATER) CC_SPEC_LAUNCH(false, 1);
                    else if (mode == MODE_LESS) CC_SPEC_LAUNCH(false, 2);
                    else CC_SPEC_LAUNCH(false, 3);
                }
#undef CC_SPEC_LAUNCH
            });
            if (lds_seams && !seams_after_fix) {
                if (ss != s) stream_wait(c, s, ss);
                seams(ss, t0, t1);
            }
        }
        launch(c, "k_params_verify", [&] {
            k_params_verify<<<grid_stride(nt), 256, 0, s>>>(g, guess, smin, smax, sflag, thr, mode, bp, TB, FIX, live);
        });
        u32* flag = c->mark.as<u32>();
        u32* list = flag + nt;
        u8* fchg = (u8*)(list + nt + 1);
        u32 nfix = 0;
        if (fast) {
            // device-gated: a fixed grid walks the k_fix list (usually empty); with the seams
            // after it nothing is marked, else it marks the seams of changed tiles and
            // k_seams_list redoes the marked ones (k_sample's front clear zeroed both)
            u8* fc_ = seams_after_fix ? nullptr : fchg;
            u32* fl_ = seams_after_fix ? nullptr : flag;
            launch(c, "k_fix", [&] {
                const unsigned grid = (unsigned)std::min<int64_t>(nt, 512);
                if (mask) k_fix_dev<true><<<grid, NTHREADS, 0, s>>>(g, FIX, bp, guess, in, mask, thr, mode, BITS, FACES, COUNT, P, KR, fc_, fl_, list);
                else k_fix_dev<false><<<grid, NTHREADS, 0, s>>>(g, FIX, bp, guess, in, nullptr, thr, mode, BITS, FACES, COUNT, P, KR, fc_, fl_, list);
            });
            if (seams_after_fix)
                seams(s, 0, nt);
            else if (lds_seams)
                launch(c, "k_seams", [&] {
                    const unsigned grid = (unsigned)std::min<int64_t>((nt + SP_WAVES - 1) / SP_WAVES, 512);
                    k_seams_list<<<grid, SP_WAVES * 64, 0, s>>>(g, FACES, COUNT, c->pairsl.as<u64>(), c->pc.as<u32>(), c->big.as<u8>(),
                                                               c->ipairs.as<u64>(), c->ipc.as<u32>(), c->iovf.as<u8>(), list);
                });
        } else {
            Readback rb(c, 64);
            rb.add(&nfix, FIX, sizeof(u32));
            rb.wait(false);
        }
        st.n_fix = nfix;
        if (lds_seams && ss != s) stream_wait(c, ss, s);
        if (nfix) {
            // one workgroup per listed tile (the same kernel as the device-gated launch, whose
            // loop then runs once); it marks the seams of the tiles whose faces changed
            HIP_OK(hipMemsetAsync(fchg, 0, nt, s));
            HIP_OK(hipMemsetAsync(flag, 0, (nt + 1) * sizeof(u32), s));
            launch(c, "k_fix", [&] {
                if (mask) k_fix_dev<true><<<nfix, NTHREADS, 0, s>>>(g, FIX, bp, guess, in, mask, thr, mode, BITS, FACES, COUNT, P, KR, fchg, flag, list);
                else k_fix_dev<false><<<nfix, NTHREADS, 0, s>>>(g, FIX, bp, guess, in, nullptr, thr, mode, BITS, FACES, COUNT, P, KR, fchg, flag, list);
            });
            if (lds_seams) {
                // relabelled faces: the seams of the relabelled tiles and of the tiles above /
                // beside them again (their lists are overwritten; stale overflow flags only send
                // work to the global fallback, which reads the current faces)
                const int64_t nl = std::min<int64_t>(nt, 14 * (int64_t)nfix);
                launch(c, "k_seams", [&] {
                    k_seams<0><<<(unsigned)((nl + SP_WAVES - 1) / SP_WAVES), SP_WAVES * 64, 0, s>>>(
                        g, FACES, COUNT, c->pairsl.as<u64>(), c->pc.as<u32>(), c->big.as<u8>(), c->ipairs.as<u64>(),
                        c->ipc.as<u32>(), c->iovf.as<u8>(), 0, 0, list);
                });
            }
        }
    }
    u8* big = c->big.as<u8>();
    u32* seg_start = c->seg.as<u32>();
    u32* seg_end = seg_start + nb;
    u64* values = c->values.as<u64>();
    u64* offsets = c->offsets.as<u64>();
    u64* scalars = c->scalars.as<u64>();
    auto ensure_roots = [&](int64_t nr) {
        c->keys.ensure(std::max<int64_t>(1, nr) * sizeof(u64));
        c->keys2.ensure(std::max<int64_t>(1, nr) * sizeof(u64));
        c->vals.ensure(std::max<int64_t>(1, nr) * sizeof(u32));
        c->vals2.ensure(std::max<int64_t>(1, nr) * sizeof(u32));
    };
    const bool block_uf = !(c->debug & CC_DEBUG_GLOBAL_STITCH);
    // k_block_uf also ranks each block's roots in first-voxel order (RL / RCB); that ranking is
    // complete unless some block took the global fallback (big[nb])
    c->rl.ensure((size_t)nb * SB_LCAP * sizeof(u32));
    c->rcb.ensure(2 * nb * sizeof(u32));
    u32* RL = c->rl.as<u32>();
    u32* RCB = c->rcb.as<u32>();
    u32* ROFFB = RCB + nb;
    if (block_uf) {
        launch(c, "k_block_uf", [&] {
            k_block_uf<<<(unsigned)nb, SB_THREADS, 0, s>>>(g, COUNT, c->pairsl.as<u64>(), c->pc.as<u32>(), P, KR, big, RL, RCB);
        });
    }
    // one mid-run host read: whether any block took the fallback, the number of roots (it sizes
    // the root arrays / LUT) and whether any tile's block-face pair list overflowed (iovf[nt]: the
    // block-face fallback k_stitch<true> is launched only then)
    u8 any_big = 1;
    u64 nr_blocks = 0;
    st.any_iovf = true;
    if (fast) {
        // no read-back: the root arrays get the context's capacity, k_block_scan flags a run that
        // needs more (RF_ROOTS) or the global fallback (RF_BIG); phase_final reads the flags
        CC_REQUIRE(block_uf, "the one-read-back schedule needs the LDS block union-find");
        // (CC_ROOT_CAP: test hook, a context's first capacity)
        if (c->root_cap == 0) c->root_cap = (uint64_t)env_int("CC_ROOT_CAP", std::max<int64_t>(1 << 16, 4 * nt));
        const uint64_t cap = c->root_cap;
        st.nr = (int64_t)cap;
        ensure_roots((int64_t)cap);
        if (nb <= SCAN_EMIT_MAXB) {
            launch(c, "k_scan_emit", [&] {
                k_scan_emit<<<(unsigned)nb, 256, 0, s>>>(nb, RL, RCB, ROFFB, values, offsets, big, scalars, cap, sum_out, KR,
                                                         c->keys2.as<u64>(), c->vals2.as<u32>(), seg_start, seg_end);
            });
        } else {
            launch(c, "k_block_scan", [&] { k_block_scan<<<1, SB_THREADS, 0, s>>>(nb, RCB, ROFFB, values, offsets, big, scalars, cap, sum_out); });
            launch(c, "k_emit_roots", [&] {
                k_emit_roots<<<(unsigned)nb, 256, 0, s>>>(RL, RCB, ROFFB, KR, offsets, c->keys2.as<u64>(), c->vals2.as<u32>(),
                                                          seg_start, seg_end, cap);
            });
        }
        st.rid0 = true;
        st.stage = 1;
        return;
    }
    CC_REQUIRE(sum_out == nullptr, "sum_out: fast schedule only");
    if (block_uf) {
        launch(c, "k_block_scan", [&] { k_block_scan<<<1, SB_THREADS, 0, s>>>(nb, RCB, ROFFB, values, offsets, big, scalars, ~0ull, nullptr); });
        u64 sc[4] = {0, 0, 0, 1};
        u8 ovf = 1;
        Readback rb(c, 64);
        rb.add(sc, scalars, 4 * sizeof(u64));             // sum of values, -, roots, "any block big" (k_block_scan)
        rb.add(&ovf, c->iovf.as<u8>() + nt, 1);
        rb.wait();
        nr_blocks = sc[2];
        any_big = sc[3] ? 1 : 0;
        st.any_iovf = ovf != 0;
        if (!any_big) {                                   // the slab's sum of block values (cc_shard_begin)
            st.sum_v = sc[0];
            st.sum_known = true;
        }
    }
    // intra-block fallback (blocks the LDS union-find could not take): only when some block needs it
    if (any_big) {
        const unsigned stitch_grid = (unsigned)std::min<int64_t>((nt + SP_WAVES - 1) / SP_WAVES, 2048);
        launch(c, "k_stitch_intra", [&] { k_stitch<false><<<stitch_grid, SP_WAVES * 64, 0, s>>>(g, FACES, P, KR, big, nullptr); });
    }
    if (!any_big) {
        const int64_t nr = (int64_t)nr_blocks;
        st.nr = nr;
        ensure_roots(nr);
        launch(c, "k_emit_roots", [&] {
            k_emit_roots<<<(unsigned)nb, 256, 0, s>>>(RL, RCB, ROFFB, KR, offsets, c->keys2.as<u64>(), c->vals2.as<u32>(),
                                                      seg_start, seg_end, ~0ull);
        });
        st.rid0 = true;
        st.stage = 1;
        return;
    }

    // generic path (some block was stitched in global memory): block-local roots of every tile
    // -> per-tile counts -> exclusive scan -> host read of the total (sizes the radix sort)
    u32* RC = c->rc.as<u32>();
    u32* ROFF = c->roff.as<u32>();
    launch(c, "k_count_roots", [&] { k_count_roots<<<grid1d(nt, WAVES), NTHREADS, 0, s>>>(g, COUNT, P, RC); });
    c->cub_tmp.ensure(prims::scan_tmp_bytes<u32>(nt + 1));
    launch(c, "scan_roots", [&] { prims::scan_excl<u32>(RC, ROFF, nt + 1, (char*)c->cub_tmp.p, s); });
    u32 n_roots_h = 0;
    {
        Readback rb(c, 64);
        rb.add(&n_roots_h, ROFF + nt, sizeof(u32));
        rb.wait();
    }
    const int64_t nr = n_roots_h;
    st.nr = nr;
    ensure_roots(nr);
    u64* keys = c->keys.as<u64>();
    u64* keys2 = c->keys2.as<u64>();
    u32* vals = c->vals.as<u32>();
    u32* vals2 = c->vals2.as<u32>();
    HIP_OK(hipMemsetAsync(seg_start, 0, 2 * nb * sizeof(u32), s));
    if (nr > 0) {
        launch(c, "k_collect_roots", [&] { k_collect_roots<<<grid1d(nt, WAVES), NTHREADS, 0, s>>>(g, COUNT, P, KR, ROFF, keys, vals); });
        int end_bit = KEY_BITS;
        while ((1LL << (end_bit - KEY_BITS)) < nb) ++end_bit;
        launch(c, "radix_sort", [&] { prims::sort_pairs<u64, u32>(keys, keys2, vals, vals2, nr, 0, end_bit, c->cub_tmp, s); });
        launch(c, "k_segments", [&] { k_segments<<<grid1d(nr), 256, 0, s>>>(nr, keys2, seg_start, seg_end); });
    }
    launch(c, "k_values", [&] { k_values<<<grid1d(nb), 256, 0, s>>>(nb, seg_start, seg_end, values); });
    c->cub_tmp.ensure(prims::scan_tmp_bytes<u64>(nb));
    launch(c, "scan_offsets", [&] { prims::scan_excl<u64>(values, offsets, nb, (char*)c->cub_tmp.p, s); });
    launch(c, "k_nlabels", [&] { k_nlabels<<<1, 1, 0, s>>>(nb, values, offsets, scalars); });
    st.stage = 1;
}

static uint64_t read_sum_v(cc_ctx* c) {
    if (state(c).sum_known) return state(c).sum_v;        // read back with the root count
    u64 v = 0;
    Readback rb(c, 64);
    rb.add(&v, c->scalars.p, sizeof(u64));
    rb.wait();
    state(c).sum_v = v;
    return v;
}

static void rid_unions(cc_ctx* c);

// global ids: offsets += base; rank -> rid; 6-connected unions across block faces
static void phase_rid(cc_ctx* c, uint64_t base) {
    RunState& st = state(c);
    CC_REQUIRE(st.stage == 1, "phase order: call begin first");
    Geom& g = st.hg.g;
    hipStream_t s = cstream(c);
    const int64_t nb = g.n_blocks, nr = st.nr;
    st.base = base;
    u64* offsets = c->offsets.as<u64>();
    if (base) launch(c, "k_add_base", [&] { k_add_base<<<grid1d(nb), 256, 0, s>>>(nb, offsets, base); });
    if (nr > 0 && !(st.rid0 && base == 0))
        launch(c, "k_assign_rid", [&] {
            k_assign_rid<<<grid1d(nr), 256, 0, s>>>(nr, c->keys2.as<u64>(), c->vals2.as<u32>(), c->seg.as<u32>(),
                                                    offsets, c->KR.as<u64>());
        });
    rid_unions(c);
}

// shards of the one-read-back schedule: the ids stay this slab's own (base 0) -- the unions are
// keyed by id order, which a common base does not change -- and the kernels after the sums'
// allgather add the base (the sums of the slabs below) themselves
static void phase_rid_dev(cc_ctx* c, const uint64_t* sums, int rank) {
    RunState& st = state(c);
    CC_REQUIRE(st.stage == 1 && st.fast, "phase order: call cc_shard_dev_begin first");
    st.base_dev = true;
    st.base = 0;
    st.sums = sums;
    st.rank = rank;
    rid_unions(c);
}

// 6-connected unions across the block faces of this volume / slab (and the empty-job emulation)
static void rid_unions(cc_ctx* c) {
    RunState& st = state(c);
    Geom& g = st.hg.g;
    hipStream_t s = cstream(c);
    const int64_t nb = g.n_blocks, nt = g.n_tiles;
    st.identity_lut = false;
    if (!st.local_only && c->quirk_jobs > 0) {
        // reference empty-job branch (merge_assignments.py:115-123): block_faces job j owns blocks
        // j :: n_jobs (cluster_tasks.py:331); if any job found no face pair, no merge happens
        c->bflag.ensure(nb);
        HIP_OK(hipMemsetAsync(c->bflag.p, 0, nb, s));
        launch(c, "k_block_face_flags", [&] {
            k_block_face_flags<<<(unsigned)((nt + 3) / 4), 256, 0, s>>>(g, c->faces.as<face_t>(), c->bflag.as<u8>());
        });
        std::vector<u8> fl(nb);
        HIP_OK(hipMemcpyAsync(fl.data(), c->bflag.p, nb, hipMemcpyDeviceToHost, s));
        sync(c);
        const int64_t nj = std::min<int64_t>(nb, c->quirk_jobs);
        for (int64_t j = 0; j < nj && !st.identity_lut; ++j) {
            bool has = false;
            for (int64_t b = j; b < nb && !has; b += nj) has = fl[b] != 0;
            st.identity_lut = !has;
        }
    }
    if (!st.local_only && !st.identity_lut) {
        launch(c, "k_inter_union", [&] {
            const int tpw = nt >= 65536 ? 64 : 16;
            k_inter_union<<<(unsigned)((nt + 4 * tpw - 1) / (4 * tpw)), 256, 0, s>>>(
                g, c->ipairs.as<u64>(), c->ipc.as<u32>(), c->P.as<u32>(), c->KR.as<u64>(), tpw,
                st.fast ? c->iovf.as<u8>() + nt : nullptr, c->scalars.as<u64>());
        });
        // tiles whose block-face pairs overflowed their list (and every tile under CC_DEBUG_GLOBAL_STITCH):
        // the global-memory fallback, in the synchronised schedule only (the one-read-back schedule
        // raises RF_IOVF in k_inter_union and the run is redone)
        if (!st.fast && st.any_iovf)
            launch(c, "k_stitch_inter", [&] {
                k_stitch<true><<<(unsigned)std::min<int64_t>((nt + SP_WAVES - 1) / SP_WAVES, 2048), SP_WAVES * 64, 0, s>>>(
                    g, c->faces.as<face_t>(), c->P.as<u32>(), c->KR.as<u64>(), c->big.as<u8>(), c->iovf.as<u8>());
            });
    }
    st.n_map = 0;
    st.stage = 2;
}

// seam planes of a slab (bottom: first voxel plane, top: last), Y*X ids each
static void phase_planes(cc_ctx* c, uint64_t* bottom, uint64_t* top) {
    RunState& st = state(c);
    CC_REQUIRE(st.stage == 2 && !st.local_only, "phase order: call assign first");
    Geom& g = st.hg.g;
    hipStream_t s = cstream(c);
    const unsigned nlayer = (unsigned)((int64_t)g.nt[1] * g.nt[2]);
    if (bottom)
        launch(c, "k_plane_labels", [&] { k_plane_labels<false><<<nlayer, NTHREADS, 0, s>>>(g, c->faces.as<face_t>(), c->P.as<u32>(), c->KR.as<u64>(), bottom); });
    if (top)
        launch(c, "k_plane_labels", [&] { k_plane_labels<true><<<nlayer, NTHREADS, 0, s>>>(g, c->faces.as<face_t>(), c->P.as<u32>(), c->KR.as<u64>(), top); });
}

// sort (a, b) pairs lexicographically and drop duplicates; pa/pb are inputs (clobbered),
// results in qa/qb; returns the number of unique pairs (host sync).  max_id: an upper bound of
// every id (~0 = unknown).  Ids below 2^32 are packed into one key a << nb | b (nb = bit width of
// max_id): one radix sort over 2 nb bits and one unique, instead of two 64-bit sorts and a flag pass.
static int64_t dedup_pairs(cc_ctx* c, u64* pa, u64* pb, u64* qa, u64* qb, int64_t n, uint64_t max_id = ~0ull) {
    hipStream_t s = cstream(c);
    if (n == 0) return 0;
    CC_REQUIRE(n < (1LL << 31), "too many pairs for one sort");
    c->scalars2.ensure(16);
    int* nsel = (int*)c->scalars2.p;
    if (max_id < (1ull << 32) && n <= prims::SU_MAX) {
        // a few thousand pairs: one workgroup packs, sorts, dedups and unpacks them in LDS
        int nbits = 1;
        while (nbits < 32 && (max_id >> nbits)) ++nbits;
        prims::k_pairs_sort_unique_small<<<1, prims::SU_T, 0, s>>>(pa, pb, (int)n, nbits, nullptr, 0, qa, qb, nsel);
        HIP_OK(hipGetLastError());
    } else if (max_id < (1ull << 32)) {
        int nbits = 1;
        while (nbits < 32 && (max_id >> nbits)) ++nbits;
        u64* k0 = qa;            // qa / qb are free until the unpack
        u64* k1 = qb;
        k_pack_pairs<<<grid1d(n), 256, 0, s>>>(n, pa, pb, nbits, k0);
        HIP_OK(hipGetLastError());
        prims::sort_keys<u64>(k0, k1, n, 0, 2 * nbits, c->cub_tmp, s);
        prims::select_unique<u64>(k1, pa, nsel, n, c->cub_tmp, s);
        k_unpack_pairs<<<grid1d(n), 256, 0, s>>>(nsel, pa, nbits, qa, qb);
        HIP_OK(hipGetLastError());
    } else {
        prims::sort_pairs<u64, u64>(pb, qb, pa, qa, n, 0, 64, c->cub_tmp, s);
        prims::sort_pairs<u64, u64>(qa, pa, qb, pb, n, 0, 64, c->cub_tmp, s);
        c->flags.ensure(n + 16);
        u8* flags = c->flags.as<u8>();
        k_unique_flags<<<grid1d(n), 256, 0, s>>>(n, pa, pb, flags);
        HIP_OK(hipGetLastError());
        prims::select_flagged<u64>(pa, flags, qa, nsel, n, c->cub_tmp, s);
        prims::select_flagged<u64>(pb, flags, qb, nsel, n, c->cub_tmp, s);
    }
    int nu = 0;
    Readback rb(c, 64);
    rb.add(&nu, nsel, sizeof(int));
    rb.wait();
    return nu;
}

// replicated union-find over the seam pairs of all slabs -> sorted id -> representative map
static void phase_map(cc_ctx* c, const u64* pairs, int64_t n) {
    RunState& st = state(c);
    CC_REQUIRE(st.stage == 2, "phase order");
    hipStream_t s = cstream(c);
    st.n_map = 0;
    if (n <= 0) return;
    // distinct ids
    c->map_ids.ensure(2 * n * sizeof(u64));
    c->map_ids2.ensure(2 * n * sizeof(u64));
    u64* ids = c->map_ids.as<u64>();
    u64* ids2 = c->map_ids2.as<u64>();
    c->scalars2.ensure(16);
    int* nsel = (int*)c->scalars2.p;
    int m = 0;
    u64 id_max = 0;
    if (2 * n <= prims::SU_MAX) {
        // a few thousand ids: the whole map (distinct ids, unions, representatives) in one
        // workgroup in LDS
        c->map_vals.ensure(2 * n * sizeof(u64));
        launch(c, "k_seam_map_small", [&] {
            prims::k_seam_map_small<<<1, prims::SU_T, 0, s>>>(pairs, (int)n, ids, c->map_vals.as<u64>(), nsel);
        });
        {
            Readback rb(c, 64);
            rb.add(&m, nsel, sizeof(int));
            rb.wait();
        }
        st.n_map = m;
        return;
    } else {
        unsigned long long* dmax = (unsigned long long*)c->scalars2.p + 1;
        HIP_OK(hipMemsetAsync(dmax, 0, sizeof(u64), s));
        launch(c, "k_copy_max64", [&] { k_copy_max64<<<grid_stride(2 * n), 256, 0, s>>>(2 * n, pairs, ids, dmax); });
        {
            Readback rb(c, 64);
            rb.add(&id_max, dmax, sizeof(u64));
            rb.wait();
        }
        int nbits = 1;
        while (nbits < 64 && (id_max >> nbits)) ++nbits;
        launch(c, "seam_sort", [&] { prims::sort_keys<u64>(ids, ids2, 2 * n, 0, nbits, c->cub_tmp, s); });
        launch(c, "seam_unique", [&] { prims::select_unique<u64>(ids2, ids, nsel, 2 * n, c->cub_tmp, s); });
    }
    {
        Readback rb(c, 64);
        rb.add(&m, nsel, sizeof(int));
        rb.wait();
    }
    if (std::getenv("CC_DEBUG_SIZES"))       // dev hook: sizes of the seam schedule
        std::fprintf(stderr, "[cc] phase_map pairs %lld ids %d max_id %llu\n", (long long)n, m, (unsigned long long)id_max);
    // U = ids[0:m]; index pairs; union-find (smallest index = smallest id) -> V
    c->map_vals.ensure(std::max<int64_t>(1, m) * sizeof(u64));
    u64* ip = ids2;    // 2n indices
    launch(c, "k_pairs_to_index", [&] { k_pairs_to_index<<<grid1d(2 * n), 256, 0, s>>>(n, pairs, ids, m, ip); });
    c->map_par.ensure(std::max<int64_t>(1, m) * sizeof(u64));
    u64* par = c->map_par.as<u64>();
    c->counter.ensure(sizeof(u32));
    HIP_OK(hipMemsetAsync(c->counter.p, 0, sizeof(u32), s));
    launch(c, "k_iota64", [&] { k_iota64<<<grid1d(m), 256, 0, s>>>((u64)m, par); });
    launch(c, "k_union_pairs", [&] { k_union_pairs<<<grid1d(n), 256, 0, s>>>(n, ip, (u64)m, par, c->counter.as<u32>()); });
    launch(c, "k_resolve64", [&] { k_resolve64<<<grid1d(m), 256, 0, s>>>((u64)m, par); });
    launch(c, "k_map_values", [&] { k_map_values<<<grid1d(m), 256, 0, s>>>(m, ids, par, c->map_vals.as<u64>()); });
    st.n_map = m;
}

// the seam map of the one-read-back shard schedule: every slab's pair buffer on the device
struct SeamDev {
    const u64* all = nullptr;   // [world][cap + 1][2]: (count, flags), then the pairs
    int world = 0;
    uint64_t cap = 0;
    const u64* sums = nullptr;  // [world] sums of block values
};

// LUT, final label per node, bit rows -> uint64 labels; small artefacts to host
static void phase_final(cc_ctx* c, uint64_t* out, cc_result* res, const SeamDev* sd = nullptr) {
    RunState& st = state(c);
    CC_REQUIRE(st.stage == 2, "phase order: call assign first");
    require_row_aligned(out, st.hg.g.X * 8);
    Geom& g = st.hg.g;
    hipStream_t s = cstream(c);
    const int64_t nt = g.n_tiles, nb = g.n_blocks, nr = st.nr;
    const uint64_t nodes = (uint64_t)nt * g.cap;
    u32* P = c->P.as<u32>();
    u64* KR = c->KR.as<u64>();
    u32* COUNT = c->count.as<u32>();
    u64* offsets = c->offsets.as<u64>();
    u64* scalars = c->scalars.as<u64>();
    const u64* U = st.n_map ? c->map_ids.as<u64>() : nullptr;
    const u64* V = st.n_map ? c->map_vals.as<u64>() : nullptr;
    const int64_t m = st.n_map;
    u64* FIN = KR;
    const uint64_t lut_cap = (uint64_t)nr + (uint64_t)nb + 1;
    StatusArgs sa;           // the one read-back's status (k_status)
    HashMap hm;
    if (sd) {
        // seam map over every slab's pairs: slots for all their ids at <= 1/4 load (cleared by this
        // step's front clear (k_sample) unless its size changed)
        CC_REQUIRE(st.fast && st.base_dev, "phase order: the device seam map follows cc_shard_dev_assign");
        uint64_t hc = 1024;
        while (hc < 8 * (uint64_t)sd->world * sd->cap) hc <<= 1;
        CC_REQUIRE(hc <= (1ull << 31), "seam map too large");
        c->hmap_keys.ensure(hc * sizeof(u64));
        c->hmap_par.ensure(hc * sizeof(u32));
        hm.keys = c->hmap_keys.as<u64>();
        hm.par = c->hmap_par.as<u32>();
        hm.mask = (u32)(hc - 1);
        if (c->hm_slots != hc) {
            launch(c, "k_map_clear", [&] { k_map_clear<<<(unsigned)std::min<uint64_t>(1024, (hc + 255) / 256), 256, 0, s>>>(hm); });
            c->hm_slots = hc;
        }
        launch(c, "k_map_build", [&] {
            k_map_build<<<(unsigned)std::min<uint64_t>(1024, (sd->world * sd->cap + 255) / 256), 256, 0, s>>>(hm, sd->all, sd->world, sd->cap);
        });
    }
    if (st.local_only) {
        c->FIN.ensure(nodes * sizeof(u64));
        FIN = c->FIN.as<u64>();
        launch(c, "k_finalize", [&] { k_finalize<true><<<grid1d(nt, WAVES), NTHREADS, 0, s>>>(g, COUNT, P, KR, offsets, U, V, m, FIN); });
        c->lut_valid = false;
    } else {
        c->lut.ensure(lut_cap * sizeof(u64));
        u64* lut = c->lut.as<u64>();
        const u64 base = st.base;
        if (st.fast) {
            c->status.ensure((16 + 2 * (size_t)nb) * sizeof(u64));
            sa.out = c->status.as<u64>();
            sa.FIX = c->spec.as<u32>() + 4 * nt + 4 * SAMPLE_PARTS * nb;
            sa.values = c->values.as<u64>();
            sa.offsets = offsets;
            sa.nb = nb;
            if (sd) { sa.all = sd->all; sa.world = sd->world; sa.cap = sd->cap; }
        }
        launch(c, "k_lut_all", [&] {
            // one workgroup per block (the id count scalars[0] + 1 stays on the device)
            k_lut_all<<<(unsigned)std::min<int64_t>(nb, 1024), 256, 0, s>>>(
                lut_cap, nb, base, st.base_dev ? st.sums : nullptr, st.rank, offsets, c->values.as<u64>(), c->seg.as<u32>(),
                c->vals2.as<u32>(), (u64)nr, P, KR, U, V, m, hm, lut, scalars);
        });
        // (the status stays a launch of its own: folded into k_pass2's last workgroup it made
        // k_pass2 0.11 ms slower at C3, profiles/r04_ab_kspec.txt)
        if (sa.out)
            launch(c, "k_status", [&] { k_status<<<1, 256, 0, s>>>(sa, scalars, st.base_dev ? st.sums : nullptr, st.rank); });
        c->lut_valid = true;
    }
    // the fused path resolves each tile component's final label inside k_pass2 (no k_finalize)
    launch(c, "k_pass2", [&] {
        // tile order of the write pass (see k_pass2): z fastest for rows of >= 4096 voxels,
        // XCD-contiguous for label rows that are not 128-B aligned (CC_PASS2_ORDER = 0 / 1 / 2
        // forces one, A/B only)
        // (and XCD-contiguous for masked volumes: C4 k_pass2 5.68-5.74 -> 5.63 ms,
        // profiles/r05_ab_c4_order_mask.txt; C3 unmasked is slower that way, 5.49-5.53 -> 5.70)
        int order = g.X >= 4096 ? 1 : ((g.X & 15) || st.masked) ? 2 : 0;
        if (const char* e = std::getenv("CC_PASS2_ORDER"); e && *e) order = std::min(std::max(std::atoi(e), 0), 5);
        // CC_LDS_PAD_P2 (A/B only): extra dynamic LDS per workgroup, i.e. fewer tiles per CU
        const unsigned pad = (unsigned)env_int("CC_LDS_PAD_P2", 0);
        // with a seam map every label goes through the slab's LUT (m = 1)
        const int64_t mm = sd ? 1 : m;
        if (st.local_only) k_pass2<false><<<(unsigned)nt, NTHREADS, pad, s>>>(g, c->bits.as<u64>(), COUNT, FIN, nullptr, nullptr, 0, 0, out, order, nullptr, nullptr);
        else k_pass2<true><<<(unsigned)nt, NTHREADS, pad, s>>>(g, c->bits.as<u64>(), COUNT, KR, P, c->lut.as<u64>(), st.base, mm, out, order,
                                                               nullptr, sd ? scalars : nullptr, lut_cap);
    });

    u64 sc[4] = {0, 0, 0, 0};
    c->h_values.resize(nb);
    c->h_offsets.resize(nb);
    st.redo = 0;
    uint64_t total = 0;
    if (st.fast) {
        // the one read-back of the run: flags, counts and the block values / offsets, gathered by
        // k_status into one buffer, one copy
        const size_t nst = 16 + 2 * (size_t)nb;
        u64* stat = c->status.as<u64>();
        std::vector<u64> h(nst);
        {
            Readback rb(c, nst * sizeof(u64) + 64);
            rb.add(h.data(), stat, nst * sizeof(u64));
            rb.wait();
        }
        st.redo = h[0];
        st.n_pairs_max = h[1];
        total = h[2];
        if (st.base_dev) st.base = h[3];
        st.n_fix = h[4];
        for (int k = 0; k < 4; ++k) sc[k] = h[5 + k];
        std::memcpy(c->h_values.data(), h.data() + 16, nb * sizeof(u64));
        std::memcpy(c->h_offsets.data(), h.data() + 16 + nb, nb * sizeof(u64));
    } else {
        Readback rb(c, 4 * sizeof(u64) + 2 * nb * sizeof(u64) + 64);
        rb.add(sc, scalars, 4 * sizeof(u64));
        rb.add(c->h_values.data(), c->values.p, nb * sizeof(u64));
        rb.add(c->h_offsets.data(), offsets, nb * sizeof(u64));
        rb.wait();
    }
    st.sum_v = sc[0];
    st.stage = 3;
    c->n_blocks = nb;
    c->n_labels = sc[0] + 1;        // LUT length of this volume (slab): ids base .. base + sum_v
    if (res) {
        res->n_blocks = nb;
        res->n_labels = sd ? total + 1 : st.base + sc[0] + 1;   // global (every slab: the allgathered sums)
        res->max_id = res->n_labels - 1;       // lut[n_labels-1] = n_labels-1 is never merged
        res->n_components = st.local_only ? 0 : sc[1];
        res->n_block_components = st.fast ? sc[2] : (uint64_t)nr;
        res->n_relabelled_tiles = st.n_fix;
        res->identity_lut = st.identity_lut ? 1 : 0;
    }
}

// The default schedule of a single volume: every launch of the five stages is enqueued without
// a host read-back (the k_fix count, the root count and the fallback flags stay on the device;
// the root arrays get the context's capacity) and the run ends in ONE read-back (k_status).
// If that read-back says the run needed more than the optimistic launch sequence covers -- the
// global-stitch fallback of a block (RF_BIG) or more roots than the capacity (RF_ROOTS) -- the
// volume is labelled again by the host-synchronised schedule, which sizes everything from
// read-back counts; the output is fully rewritten, so which schedule ran never shows in the
// result.  CC_FAST=0 (A/B, tests) forces the host-synchronised schedule.
static bool fast_ok(cc_ctx* c) {
    if (c->debug & CC_DEBUG_GLOBAL_STITCH) return false;
    if (c->quirk_jobs > 0 || c->front_chunks > 1) return false;
    return env_int("CC_FAST", 1) != 0;
}

static void run_pipeline(cc_ctx* c, const float* in, const uint8_t* mask, const int64_t shape[3],
                         const int64_t block_shape[3], double threshold, int mode, uint64_t* out,
                         bool local_only, cc_result* res) {
    if (!local_only && fast_ok(c)) {
        const HostGeom hg = make_geom(shape, block_shape, 0);
        // a volume of this geometry needed the fallback last time: go synchronised directly
        if (!(c->fast_big && c->fast_big_tab == hg.tab)) {
            phase_local(c, in, mask, shape, block_shape, threshold, mode, 0, false, true);
            phase_rid(c, 0);
            phase_final(c, out, res);
            const uint64_t redo = state(c).redo;
            if (!redo) {
                c->fast_big = false;
                return;
            }
            // a block needing the global stitch or a tile's overflowed block-face pair list are
            // properties of the input: the next volume of this geometry goes synchronised directly
            c->fast_big = (redo & (RF_BIG | RF_IOVF)) != 0;
            if (c->fast_big) c->fast_big_tab = hg.tab;
        }
    }
    phase_local(c, in, mask, shape, block_shape, threshold, mode, 0, local_only);
    phase_rid(c, 0);
    phase_final(c, out, res);
    // the next optimistic run of this context gets room for this many roots
    if (!state(c).local_only) c->root_cap = std::max<uint64_t>(c->root_cap, (uint64_t)state(c).nr + (uint64_t)state(c).nr / 4 + 1024);
}

// ------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------
extern "C" {

#ifndef CC_SRC_HASH
#define CC_SRC_HASH "unknown"
#endif
// "src=" carries the SHA-256 prefix of the sources this library was built from (build.py)
const char* cc_version(void) { return "cc_mi355x 0.2 gfx950 src=" CC_SRC_HASH; }

const char* cc_last_error(void) { return g_err.c_str(); }

int64_t cc_result_size(void) { return (int64_t)sizeof(cc_result); }

int cc_create(int device, cc_ctx** out) {
    CC_TRY({
        CC_REQUIRE(out != nullptr, "out is NULL");
        int n = 0;
        HIP_OK(hipGetDeviceCount(&n));
        CC_REQUIRE(device >= 0 && device < n, "no such HIP device");
        HIP_OK(hipSetDevice(device));
        cc_ctx* c = new cc_ctx();
        c->device = device;
        if (const char* e = std::getenv("CC_FRONT_CHUNKS")) c->front_chunks = std::max(1, atoi(e));
        for (DevBuf* b : ctx_bufs(c)) b->stream = &c->stream;   // released pieces wait for this stream's work
        *out = c;
    })
}

void cc_destroy(cc_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    if (c->side) (void)hipStreamSynchronize(c->side);
    for (DevBuf* b : ctx_bufs(c)) b->release();
    c->pin.release();
    g_arena.trim();             // the stream has drained: the context's pieces are free again
    for (auto& pe : c->pending) { (void)hipEventDestroy(pe.second.first); (void)hipEventDestroy(pe.second.second); }
    for (hipEvent_t e : c->event_pool) (void)hipEventDestroy(e);
    if (c->side) (void)hipStreamDestroy(c->side);
    delete (RunState*)c->run;
    delete c;
}

int cc_set_stream(cc_ctx* c, void* stream) {
    CC_TRY({
        CC_REQUIRE(c, "ctx is NULL");
        // the context's buffers are released behind events on its stream: work still queued on
        // the previous stream must be done before another stream takes over
        if (c->stream != (hipStream_t)stream) {
            HIP_OK(hipSetDevice(c->device));
            HIP_OK(hipStreamSynchronize(c->stream));
            if (c->side) HIP_OK(hipStreamSynchronize(c->side));
        }
        c->stream = (hipStream_t)stream;
    })
}

int cc_label_volume(cc_ctx* c, const float* in, const uint8_t* mask, const int64_t shape[3],
                    const int64_t block_shape[3], double threshold, int mode, uint64_t* labels,
                    cc_result* res) {
    CC_TRY({
        CC_REQUIRE(c && in && labels && shape && block_shape, "NULL argument");
        HIP_OK(hipSetDevice(c->device));
        run_pipeline(c, in, mask, shape, block_shape, threshold, to_mode(mode), labels, false, res);
    })
}

int cc_label_volume_host(cc_ctx* c, const float* in, const uint8_t* mask, const int64_t shape[3],
                         const int64_t block_shape[3], double threshold, int mode, uint64_t* labels,
                         cc_result* res) {
    CC_TRY({
        CC_REQUIRE(c && in && labels && shape && block_shape, "NULL argument");
        HIP_OK(hipSetDevice(c->device));
        const int64_t n = shape[0] * shape[1] * shape[2];
        c->in_tmp.ensure(n * sizeof(float));
        c->out_tmp.ensure(n * sizeof(u64));
        HIP_OK(hipMemcpyAsync(c->in_tmp.p, in, n * sizeof(float), hipMemcpyHostToDevice, cstream(c)));
        const uint8_t* dmask = nullptr;
        if (mask) {
            c->mask_tmp.ensure(n);
            HIP_OK(hipMemcpyAsync(c->mask_tmp.p, mask, n, hipMemcpyHostToDevice, cstream(c)));
            dmask = c->mask_tmp.as<uint8_t>();
        }
        run_pipeline(c, c->in_tmp.as<float>(), dmask, shape, block_shape, threshold, to_mode(mode),
                     c->out_tmp.as<uint64_t>(), false, res);
        HIP_OK(hipMemcpyAsync(labels, c->out_tmp.p, n * sizeof(u64), hipMemcpyDeviceToHost, cstream(c)));
        sync(c);
    })
}

int64_t cc_get_block_values(cc_ctx* c, uint64_t* out, int64_t cap) {
    if (!c || !out) { g_err = "NULL argument"; return -1; }
    if (cap < (int64_t)c->h_values.size()) { g_err = "cap too small"; return -1; }
    std::memcpy(out, c->h_values.data(), c->h_values.size() * sizeof(uint64_t));
    return (int64_t)c->h_values.size();
}

int64_t cc_get_offsets(cc_ctx* c, uint64_t* out, int64_t cap) {
    if (!c || !out) { g_err = "NULL argument"; return -1; }
    if (cap < (int64_t)c->h_offsets.size()) { g_err = "cap too small"; return -1; }
    std::memcpy(out, c->h_offsets.data(), c->h_offsets.size() * sizeof(uint64_t));
    return (int64_t)c->h_offsets.size();
}

int64_t cc_get_lut(cc_ctx* c, uint64_t* out, int64_t cap) {
    if (!c || !out) { g_err = "NULL argument"; return -1; }
    if (!c->lut_valid) { g_err = "no LUT: run cc_label_volume first"; return -1; }
    if (cap < (int64_t)c->n_labels) { g_err = "cap too small"; return -1; }
    try {
        HIP_OK(hipSetDevice(c->device));
        HIP_OK(hipMemcpyAsync(out, c->lut.p, c->n_labels * sizeof(u64), hipMemcpyDeviceToHost, cstream(c)));
        sync(c);
    } catch (const CCError& e) {
        g_err = e.msg;
        return -1;
    }
    return (int64_t)c->n_labels;
}

int cc_block_components(cc_ctx* c, const float* in, const uint8_t* mask, const int64_t shape[3],
                        const int64_t block_shape[3], double threshold, int mode, uint64_t* labels,
                        uint64_t* values_host, int64_t n_blocks) {
    CC_TRY({
        CC_REQUIRE(c && in && labels && shape && block_shape, "NULL argument");
        HIP_OK(hipSetDevice(c->device));
        run_pipeline(c, in, mask, shape, block_shape, threshold, to_mode(mode), labels, true, nullptr);
        if (values_host) {
            CC_REQUIRE(n_blocks >= c->n_blocks, "values buffer too small");
            std::memcpy(values_host, c->h_values.data(), c->n_blocks * sizeof(uint64_t));
        }
    })
}

int cc_threshold(cc_ctx* c, const float* in, const int64_t shape[3], const int64_t block_shape[3],
                 double threshold, int mode, uint8_t* out) {
    CC_TRY({
        CC_REQUIRE(c && in && out && shape && block_shape, "NULL argument");
        require_row_aligned(in, shape[2] * 4);
        HIP_OK(hipSetDevice(c->device));
        const int md = to_mode(mode);
        RunState& st = state(c);
        st = RunState();
        st.hg = make_geom(shape, block_shape, 0);
        upload_geom(c, st.hg);
        Geom& g = st.hg.g;
        const int64_t nt = g.n_tiles, nb = g.n_blocks;
        hipStream_t s = cstream(c);
        c->bstat.ensure(nb * 3 * sizeof(u32));
        c->bparam.ensure(2 * nb * sizeof(BlockParam));
        u32* smin = c->bstat.as<u32>();
        u32* smax = smin + nb;
        u32* sflag = smax + nb;
        BlockParam* bp = c->bparam.as<BlockParam>();
        BlockParam* guess = bp + nb;
        const float thr = (float)threshold;          // numpy: python float -> float32
        if (const char* e = std::getenv("CC_THRESHOLD_TWO_PASS"); e && std::string(e) == "1") {
            // A/B only: statistics pass, then the threshold pass (two reads of the input)
            HIP_OK(hipMemsetAsync(smin, 0xFF, nb * sizeof(u32), s));
            HIP_OK(hipMemsetAsync(smax, 0x00, 2 * nb * sizeof(u32), s));
            launch(c, "k_block_stats", [&] { k_block_stats<<<(unsigned)nt, NTHREADS, 0, s>>>(g, in, smin, smax, sflag); });
            launch(c, "k_block_params", [&] {
                k_block_params<<<(unsigned)((nb + 255) / 256), 256, 0, s>>>(nb, smin, smax, sflag, thr, md, bp);
            });
            launch(c, "k_threshold", [&] { k_threshold<<<(unsigned)nt, NTHREADS, 0, s>>>(g, bp, in, thr, md, out); });
        } else {
            // one read: sample -> guessed interval -> threshold + exact statistics + TB per tile ->
            // exact parameters, list of tiles whose guessed output is not exact -> rewrite those
            c->spec.ensure((4 * nt + 4 * SAMPLE_PARTS * nb + nt + 1) * sizeof(u32));
            u32* TB = c->spec.as<u32>();
            u32* SPART = TB + 4 * nt;
            u32* FIX = SPART + 4 * SAMPLE_PARTS * nb;
            HIP_OK(hipMemsetAsync(smin, 0xFF, nb * sizeof(u32), s));
            HIP_OK(hipMemsetAsync(smax, 0x00, 2 * nb * sizeof(u32), s));
            HIP_OK(hipMemsetAsync(FIX, 0, sizeof(u32), s));
            FrontClear none{};
            launch(c, "k_sample", [&] { k_sample<<<(unsigned)(nb * SAMPLE_PARTS), NTHREADS, 0, s>>>(g, in, SPART, none); });
            launch(c, "k_guess", [&] { k_guess<<<(unsigned)((nb + 255) / 256), 256, 0, s>>>(nb, SPART, thr, md, guess); });
            if (const char* e = std::getenv("CC_SPEC"); e && std::string(e) == "0")     // test hook: no guesses
                HIP_OK(hipMemsetAsync(guess, 0, nb * sizeof(BlockParam), s));
            SpecArgs sa;
            sa.guess = guess;
            sa.smin = smin; sa.smax = smax; sa.sflag = sflag;
            sa.TB = TB;
            sa.t0 = 0;
            launch(c, "k_thr_spec", [&] {
                const unsigned ng = (unsigned)((nt + 3) / 4);       // four x-adjacent tiles per workgroup
                if (md == MODE_GREATER) k_thr_spec<1><<<ng, NTHREADS, 0, s>>>(g, sa, in, out);
                else if (md == MODE_LESS) k_thr_spec<2><<<ng, NTHREADS, 0, s>>>(g, sa, in, out);
                else k_thr_spec<3><<<ng, NTHREADS, 0, s>>>(g, sa, in, out);
            });
            launch(c, "k_params_verify", [&] {
                k_params_verify<<<grid_stride(nt), 256, 0, s>>>(g, guess, smin, smax, sflag, thr, md, bp, TB, FIX, nullptr);
            });
            launch(c, "k_thr_fix", [&] {
                k_thr_fix<<<(unsigned)std::min<int64_t>(nt, 2048), NTHREADS, 0, s>>>(g, FIX, bp, in, thr, md, out);
            });
        }
        sync(c);
        st.stage = 0;
    })
}

int cc_resize_mask_nearest(cc_ctx* c, const uint8_t* mask, const int64_t mshape[3], const int64_t shape[3],
                           int64_t z0, int64_t nz, uint8_t* out) {
    CC_TRY({
        CC_REQUIRE(c && mask && mshape && shape && out, "NULL argument");
        require_row_aligned(mask, mshape[2]);
        require_row_aligned(out, shape[2]);
        for (int a = 0; a < 3; ++a) CC_REQUIRE(mshape[a] > 0 && shape[a] > 0, "empty mask or volume");
        CC_REQUIRE(z0 >= 0 && nz >= 0 && z0 + nz <= shape[0], "z range outside the volume");
        CC_REQUIRE(shape[1] * shape[2] < (1LL << 40) && (2 * shape[2] + 1) * mshape[2] < (1LL << 62) &&
                       (2 * shape[1] + 1) * mshape[1] < (1LL << 62) && (2 * shape[0] + 1) * mshape[0] < (1LL << 62),
                   "mask / volume extents too large");
        CC_REQUIRE(nz * shape[1] < (1LL << 31), "too many rows for one launch");
        HIP_OK(hipSetDevice(c->device));
        if (nz == 0) return 0;
        hipStream_t s = cstream(c);
        // 16 bytes per thread when the rows allow 16-B stores (X % 16 == 0, out 16-B aligned)
        const bool w16 = shape[2] % 16 == 0 && ((uintptr_t)out & 15) == 0 && nz * shape[1] < (1LL << 32);
        if (w16) {
            c->mask_xmap.ensure((shape[0] + shape[1] + shape[2]) * sizeof(int32_t));
            int32_t* map = c->mask_xmap.as<int32_t>();
            launch(c, "k_mask_xmap", [&] {
                k_mask_maps<<<grid_stride(shape[0] + shape[1] + shape[2]), 256, 0, s>>>(shape[2], shape[1], shape[0], mshape[2],
                                                                                   mshape[1], mshape[0], map);
            });
            launch(c, "k_mask_resize", [&] {
                k_mask_resize16<<<grid_stride(nz * shape[1] * (shape[2] / 16)), 256, 0, s>>>(
                    mask, mshape[1], mshape[2], shape[1], shape[2], z0, nz * shape[1], map, out);
            });
        } else {
            c->mask_xmap.ensure(shape[2] * sizeof(int32_t));
            launch(c, "k_mask_xmap", [&] { k_mask_xmap<<<grid_stride(shape[2]), 256, 0, s>>>(shape[2], mshape[2], c->mask_xmap.as<int32_t>()); });
            const dim3 grid((unsigned)((shape[2] + 1023) / 1024), (unsigned)(nz * shape[1]));
            launch(c, "k_mask_resize", [&] {
                k_mask_resize<<<grid, 256, 0, s>>>(mask, mshape[0], mshape[1], mshape[2], shape[0], shape[1], shape[2], z0,
                                                   c->mask_xmap.as<int32_t>(), out);
            });
        }
        sync(c);
    })
}

int cc_merge_offsets(const uint64_t* values, int64_t n_blocks, uint64_t* offsets, uint8_t* empty,
                     uint64_t* n_labels) {
    CC_TRY({
        CC_REQUIRE(values && n_blocks > 0, "bad arguments");
        uint64_t acc = 0;
        for (int64_t b = 0; b < n_blocks; ++b) {
            if (offsets) offsets[b] = acc;
            if (empty) empty[b] = values[b] == 0;
            acc += values[b];
        }
        if (n_labels) *n_labels = acc + 1;   // offsets[-1] + values[-1] + 1
    })
}

int cc_set_profiling(cc_ctx* c, int enable) {
    CC_TRY({
        CC_REQUIRE(c, "ctx is NULL");
        CC_REQUIRE(enable >= 0 && enable <= 2, "profiling level must be 0, 1 or 2");
        c->prof = enable;
    })
}

int cc_set_option(cc_ctx* c, int option, int64_t value) {
    CC_TRY({
        CC_REQUIRE(c, "ctx is NULL");
        if (option == CC_OPT_EMPTY_JOB_QUIRK) {
            CC_REQUIRE(value >= 0, "max_jobs must be >= 0");
            c->quirk_jobs = value;
        } else if (option == CC_OPT_WS_PRENORMALIZED) {
            c->ws_prenormalized = value != 0;
        } else {
            CC_REQUIRE(false, "unknown option");
        }
    })
}

int cc_set_debug(cc_ctx* c, int flags) {
    CC_TRY({
        CC_REQUIRE(c, "ctx is NULL");
        c->debug = flags;
    })
}

int cc_reset_profile(cc_ctx* c) {
    CC_TRY({
        CC_REQUIRE(c, "ctx is NULL");
        c->prof_acc.clear();
        g_alloc_count = 0;
        g_alloc_ns = 0;
        g_sync_count = 0;
        g_sync_ns = 0;
    })
}

int cc_get_profile(cc_ctx* c, char* names, int names_cap, int64_t* counts, double* total_ms, int cap) {
    if (!c) { g_err = "ctx is NULL"; return -1; }
    std::string joined;
    int i = 0;
    std::map<std::string, ProfEntry> acc = c->prof_acc;
    if (g_alloc_count) acc["host_alloc"] = ProfEntry{g_alloc_count.load(), g_alloc_ns.load() * 1e-6};
    if (g_sync_count) acc["host_sync"] = ProfEntry{g_sync_count.load(), g_sync_ns.load() * 1e-6};
    for (auto& kv : acc) {
        if (i >= cap) break;
        if (!joined.empty()) joined += ",";
        joined += kv.first;
        if (counts) counts[i] = kv.second.count;
        if (total_ms) total_ms[i] = kv.second.ms;
        ++i;
    }
    if (names && names_cap > 0) {
        std::strncpy(names, joined.c_str(), names_cap - 1);
        names[names_cap - 1] = 0;
    }
    return i;
}

}  // extern "C"

#include "cc_stage_host.hip"
#include "cc_comm.hip"
