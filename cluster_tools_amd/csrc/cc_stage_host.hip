// cc_stage_host.hip -- host side of the stage-level entry points and the generator (included at the
// end of cc_lib.hip, same translation unit).

extern "C" {

int64_t cc_block_faces(cc_ctx* c, const uint64_t* labels, const int64_t shape[3], const int64_t block_shape[3],
                       const uint64_t* offsets_host, uint64_t* pairs_host, int64_t cap, uint8_t* block_has_pairs_host) {
    try {
        CC_REQUIRE(c && labels && shape && block_shape && offsets_host, "NULL argument");
        require_row_aligned(labels, shape[2] * 8);
        HIP_OK(hipSetDevice(c->device));
        hipStream_t s = cstream(c);
        int64_t nb[3], n_face = 0;
        for (int a = 0; a < 3; ++a) {
            CC_REQUIRE(shape[a] >= 1 && block_shape[a] >= 1, "bad shape / block_shape");
            nb[a] = (shape[a] + block_shape[a] - 1) / block_shape[a];
        }
        const int64_t n_blocks = nb[0] * nb[1] * nb[2];
        for (int a = 0; a < 3; ++a)
            n_face += ((shape[a] - 1) / block_shape[a]) * (shape[0] * shape[1] * shape[2] / shape[a]);
        c->offsets.ensure(n_blocks * sizeof(u64));
        HIP_OK(hipMemcpyAsync(c->offsets.p, offsets_host, n_blocks * sizeof(u64), hipMemcpyHostToDevice, s));
        const int64_t capn = std::max<int64_t>(1, n_face);
        c->pairs.ensure(2 * capn * sizeof(u64));
        c->pairs2.ensure(2 * capn * sizeof(u64));
        c->counter.ensure(2 * sizeof(unsigned long long));
        c->scalars.ensure(SCALARS * sizeof(u64));
        u64* pa = c->pairs.as<u64>();
        u64* pb = pa + capn;
        u64* qa = c->pairs2.as<u64>();
        u64* qb = qa + capn;
        unsigned long long* cnt = (unsigned long long*)c->counter.p;
        u8* bflag = nullptr;
        if (block_has_pairs_host) {
            c->bflag.ensure(n_blocks);
            bflag = c->bflag.as<u8>();
            HIP_OK(hipMemsetAsync(bflag, 0, n_blocks, s));
        }
        unsigned long long* maxid = cnt + 1;
        HIP_OK(hipMemsetAsync(cnt, 0, 2 * sizeof(unsigned long long), s));
        for (int a = 0; a < 3; ++a) {
            FaceGeom G;
            for (int d = 0; d < 3; ++d) { G.S[d] = shape[d]; G.B[d] = block_shape[d]; G.nb[d] = nb[d]; }
            G.axis = a;
            G.fdim = a == 2 ? 1 : 2;
            G.rdim = a == 0 ? 1 : 0;
            const int64_t nplanes = (shape[a] - 1) / block_shape[a];
            const int64_t nchunk = (shape[G.fdim] + FP_CHUNK - 1) / FP_CHUNK;
            if (nplanes == 0) continue;
            const int64_t nrowg = (shape[G.rdim] + FP_ROWS - 1) / FP_ROWS;
            CC_REQUIRE(nrowg < 65536 && nplanes < 65536 && nchunk < (1LL << 31) && shape[G.fdim] < (1LL << 32),
                       "face-pair grid out of range");
            const dim3 grid((unsigned)nchunk, (unsigned)nrowg, (unsigned)nplanes);
            launch(c, "k_face_pairs", [&] {
                k_face_pairs<<<grid, FACE_PAIR_THREADS, 0, s>>>(G, labels, c->offsets.as<u64>(), pa, pb, cnt, (u64)capn,
                                                                maxid, bflag);
            });
        }
        unsigned long long rb2[2] = {0, 0};
        HIP_OK(hipMemcpyAsync(rb2, cnt, sizeof(rb2), hipMemcpyDeviceToHost, s));
        if (bflag) HIP_OK(hipMemcpyAsync(block_has_pairs_host, bflag, n_blocks, hipMemcpyDeviceToHost, s));
        sync(c);
        const int64_t n = (int64_t)rb2[0];
        if (n == 0) return 0;
        CC_REQUIRE(n <= capn, "face pair buffer overflow");
        // lexicographic sort + unique (block_faces.py:112,132,172 np.unique(axis=0))
        const int64_t nu = dedup_pairs(c, pa, pb, qa, qb, n, (uint64_t)rb2[1]);
        if (pairs_host && cap > 0) {
            const int64_t m = std::min<int64_t>(cap, nu);
            std::vector<u64> ha(m), hb(m);
            HIP_OK(hipMemcpyAsync(ha.data(), qa, m * sizeof(u64), hipMemcpyDeviceToHost, s));
            HIP_OK(hipMemcpyAsync(hb.data(), qb, m * sizeof(u64), hipMemcpyDeviceToHost, s));
            sync(c);
            for (int64_t i = 0; i < m; ++i) { pairs_host[2 * i] = ha[i]; pairs_host[2 * i + 1] = hb[i]; }
        }
        return nu;
    } catch (const CCError& e) {
        g_err = e.msg;
        return -1;
    }
}

int cc_merge_assignments(cc_ctx* c, const uint64_t* pairs_host, int64_t n_pairs, uint64_t n_labels,
                         uint64_t* lut_host) {
    CC_TRY({
        CC_REQUIRE(c && lut_host && n_labels >= 1 && n_pairs >= 0, "bad arguments");
        CC_REQUIRE(n_pairs == 0 || pairs_host, "pairs is NULL");
        HIP_OK(hipSetDevice(c->device));
        hipStream_t s = cstream(c);
        c->lut.ensure(n_labels * sizeof(u64));
        c->pairs.ensure(std::max<int64_t>(1, 2 * n_pairs) * sizeof(u64));
        c->counter.ensure(sizeof(u32));
        u64* P = c->lut.as<u64>();
        u32* err = c->counter.as<u32>();
        HIP_OK(hipMemsetAsync(err, 0, sizeof(u32), s));
        launch(c, "k_iota64", [&] { k_iota64<<<grid1d(n_labels), 256, 0, s>>>(n_labels, P); });
        if (n_pairs > 0) {
            HIP_OK(hipMemcpyAsync(c->pairs.p, pairs_host, 2 * n_pairs * sizeof(u64), hipMemcpyHostToDevice, s));
            launch(c, "k_union_pairs", [&] {
                k_union_pairs<<<grid1d(n_pairs), 256, 0, s>>>(n_pairs, c->pairs.as<u64>(), n_labels, P, err);
            });
        }
        launch(c, "k_resolve64", [&] { k_resolve64<<<grid1d(n_labels), 256, 0, s>>>(n_labels, P); });
        u32 herr = 0;
        HIP_OK(hipMemcpyAsync(&herr, err, sizeof(u32), hipMemcpyDeviceToHost, s));
        HIP_OK(hipMemcpyAsync(lut_host, P, n_labels * sizeof(u64), hipMemcpyDeviceToHost, s));
        sync(c);
        c->n_labels = n_labels;
        c->lut_valid = true;
        CC_REQUIRE(herr == 0, "assignment id >= n_labels (merge_assignments.py:124)");
    })
}

int cc_write(cc_ctx* c, uint64_t* labels, const int64_t shape[3], const int64_t block_shape[3],
             const uint64_t* offsets_host, const uint64_t* lut_host, uint64_t n_labels) {
    CC_TRY({
        CC_REQUIRE(c && labels && shape && block_shape && offsets_host && lut_host && n_labels >= 1, "bad arguments");
        require_row_aligned(labels, shape[2] * 8);
        HIP_OK(hipSetDevice(c->device));
        hipStream_t s = cstream(c);
        int64_t nb[3];
        for (int a = 0; a < 3; ++a) nb[a] = (shape[a] + block_shape[a] - 1) / block_shape[a];
        const int64_t n_blocks = nb[0] * nb[1] * nb[2];
        const int64_t n = shape[0] * shape[1] * shape[2];
        c->offsets.ensure(n_blocks * sizeof(u64));
        c->lut.ensure(n_labels * sizeof(u64));
        c->counter.ensure(sizeof(u32));
        HIP_OK(hipMemcpyAsync(c->offsets.p, offsets_host, n_blocks * sizeof(u64), hipMemcpyHostToDevice, s));
        HIP_OK(hipMemcpyAsync(c->lut.p, lut_host, n_labels * sizeof(u64), hipMemcpyHostToDevice, s));
        HIP_OK(hipMemsetAsync(c->counter.p, 0, sizeof(u32), s));
        const int64_t nchunk = (shape[2] + WRITE_CHUNK - 1) / WRITE_CHUNK;
        CC_REQUIRE(shape[0] < 65536 && shape[1] < 65536 && shape[2] < (1LL << 32), "volume too large for the write grid");
        if (n > 0)
            launch(c, "k_write_offsets", [&] {
                k_write_offsets<<<dim3((unsigned)nchunk, (unsigned)shape[1], (unsigned)shape[0]), WRITE_THREADS, 0, s>>>(
                    shape[1], shape[2], block_shape[0], block_shape[1], (u32)block_shape[2], nb[1], nb[2], labels,
                    c->offsets.as<u64>(), c->lut.as<u64>(), n_labels, c->counter.as<u32>());
            });
        u32 herr = 0;
        HIP_OK(hipMemcpyAsync(&herr, c->counter.p, sizeof(u32), hipMemcpyDeviceToHost, s));
        sync(c);
        CC_REQUIRE(herr == 0, "label id exceeds number of node labels (write.py:164)");
    })
}

int cc_generate_boundary_map(cc_ctx* c, float* out, const int64_t shape[3], const int64_t origin[3],
                             uint64_t seed, int dither) {
    CC_TRY({
        CC_REQUIRE(c && out && shape, "NULL argument");
        require_row_aligned(out, shape[2] * 4);
        HIP_OK(hipSetDevice(c->device));
        int64_t o[3] = {0, 0, 0};
        if (origin) { o[0] = origin[0]; o[1] = origin[1]; o[2] = origin[2]; }
        for (int a = 0; a < 3; ++a) CC_REQUIRE(shape[a] >= 1 && o[a] >= 0 && o[a] + shape[a] < (1LL << 21), "bad shape/origin");
        const int64_t nxb = (shape[2] + 255) / 256;
        CC_REQUIRE(shape[1] * nxb < (1LL << 24) && shape[0] < 65536, "volume too large for the generator grid");
        const dim3 grid((unsigned)(shape[1] * nxb), (unsigned)shape[0]);
        launch(c, "k_generate", [&] {
            k_generate<<<grid, 256, 0, cstream(c)>>>(out, shape[0], shape[1], shape[2], o[0], o[1], o[2], seed, dither);
        });
        sync(c);
    })
}

}  // extern "C"

// ---------------------------------------------------------------------------------------------
// z-slab sharding (multi-GPU): see cluster_tools_amd/distributed.py for the collective schedule
// ---------------------------------------------------------------------------------------------
extern "C" {

int cc_shard_begin(cc_ctx* c, const float* in, const uint8_t* mask, const int64_t slab_shape[3],
                   const int64_t block_shape[3], double threshold, int mode, int64_t z_offset,
                   uint64_t* sum_values) {
    CC_TRY({
        CC_REQUIRE(c && in && slab_shape && block_shape && sum_values, "NULL argument");
        CC_REQUIRE(z_offset >= 0 && z_offset % block_shape[0] == 0,
                   "slab z offset must be a multiple of block_shape[0] (seams on block faces)");
        CC_REQUIRE(c->quirk_jobs == 0, "the empty-job emulation is not available on the z-slab path");
        HIP_OK(hipSetDevice(c->device));
        phase_local(c, in, mask, slab_shape, block_shape, threshold, to_mode(mode), z_offset, false);
        *sum_values = read_sum_v(c);
        // room for this many roots in the next one-read-back step of this context
        c->root_cap = std::max<uint64_t>(c->root_cap, (uint64_t)state(c).nr + (uint64_t)state(c).nr / 4 + 1024);
    })
}

int cc_shard_assign(cc_ctx* c, uint64_t id_base) {
    CC_TRY({
        CC_REQUIRE(c, "NULL ctx");
        HIP_OK(hipSetDevice(c->device));
        phase_rid(c, id_base);
    })
}

int cc_shard_planes(cc_ctx* c, uint64_t* bottom, uint64_t* top) {
    CC_TRY({
        CC_REQUIRE(c, "NULL ctx");
        HIP_OK(hipSetDevice(c->device));
        phase_planes(c, bottom, top);      // enqueued on the ctx's stream (callers order by stream)
    })
}

}  // extern "C"

template <class UP>
static int64_t seam_pairs_impl(cc_ctx* c, UP upper, const uint64_t* lower, int64_t n, uint64_t* pairs,
                               int64_t cap) {
    CC_REQUIRE(c && upper.p && lower && n >= 0, "bad arguments");
    HIP_OK(hipSetDevice(c->device));
    hipStream_t s = cstream(c);
    const int64_t capn = std::max<int64_t>(1, n);
    c->pairs.ensure(2 * capn * sizeof(u64));
    c->pairs2.ensure(2 * capn * sizeof(u64));
    c->counter.ensure(2 * sizeof(unsigned long long));
    u64* pa = c->pairs.as<u64>();
    u64* pb = pa + capn;
    u64* qa = c->pairs2.as<u64>();
    u64* qb = qa + capn;
    c->counter.ensure(4 * sizeof(unsigned long long));
    unsigned long long* cnt = (unsigned long long*)c->counter.p;
    // the pair hash set (see k_seam_pairs): 2^16 slots
    constexpr int64_t HS = 1 << 16;
    c->seam_hash.ensure(HS * sizeof(u64));
    u64* htab = c->seam_hash.as<u64>();
    HIP_OK(hipMemsetAsync(cnt, 0, 3 * sizeof(unsigned long long), s));
    HIP_OK(hipMemsetAsync(htab, 0xFF, HS * sizeof(u64), s));
    // plane width for the 'pair above' filter (any value is correct; the slab's X is exact)
    const int64_t X = (c->run && state(c).hg.g.Y * state(c).hg.g.X == n) ? state(c).hg.g.X : n;
    launch(c, "k_seam_pairs", [&] {
        k_seam_pairs<UP><<<(unsigned)((n + SP_WG_VOXELS - 1) / SP_WG_VOXELS), SEAM_PAIR_THREADS, 0, s>>>(
            n, X, upper, lower, pa, pb, cnt, (u64)capn, htab, (u32)(HS - 1));
    });
    unsigned long long rb2[3] = {0, 0, 0};       // pairs appended, largest id, flags
    {
        Readback rb(c, 64);
        rb.add(rb2, cnt, sizeof(rb2));
        rb.wait();
    }
    const unsigned long long n_raw = rb2[0];
    CC_REQUIRE(n_raw <= (unsigned long long)capn, "seam pair buffer overflow");
    int64_t nu = 0;
    if (rb2[2] == 0 && n_raw <= (unsigned long long)prims::SU_MAX) {
        // the appended pairs are distinct: one workgroup sorts them into the caller's buffer
        nu = (int64_t)n_raw;
        int nb = 1;
        while (nb < 32 && (rb2[1] >> nb)) ++nb;
        c->scalars2.ensure(16);
        if (nu > 0)
            launch(c, "seam_sort_small", [&] {
                prims::k_pairs_sort_unique_small<<<1, prims::SU_T, 0, s>>>(pa, pb, (int)nu, nb, pairs, cap, nullptr, nullptr,
                                                                          (int*)c->scalars2.p);
            });
        if (std::getenv("CC_DEBUG_SIZES"))       // dev hook: sizes of the seam schedule
            std::fprintf(stderr, "[cc] seam_pairs plane %lld unique %lld max_id %llu (hash set)\n", (long long)n,
                         (long long)nu, (unsigned long long)rb2[1]);
        return nu;
    }
    launch(c, "seam_dedup", [&] { nu = dedup_pairs(c, pa, pb, qa, qb, (int64_t)n_raw, (uint64_t)rb2[1]); });
    if (std::getenv("CC_DEBUG_SIZES"))       // dev hook: sizes of the seam schedule
        std::fprintf(stderr, "[cc] seam_pairs plane %lld raw %llu unique %lld max_id %llu\n", (long long)n,
                     n_raw, (long long)nu, (unsigned long long)rb2[1]);
    if (pairs && cap > 0 && nu > 0) {
        const int64_t m = std::min<int64_t>(cap, nu);
        launch(c, "k_interleave", [&] { k_interleave<<<grid1d(m), 256, 0, s>>>(m, qa, qb, pairs); });
        sync(c);
    }
    return nu;
}

extern "C" {

int64_t cc_seam_pairs(cc_ctx* c, const uint64_t* upper, const uint64_t* lower, int64_t n, uint64_t* pairs,
                      int64_t cap) {
    try {
        return seam_pairs_impl(c, UpperIds{upper}, lower, n, pairs, cap);
    } catch (const CCError& e) {
        g_err = e.msg;
        return -1;
    }
}

int64_t cc_seam_pairs32(cc_ctx* c, const uint32_t* upper32, uint64_t upper_base, const uint64_t* lower, int64_t n,
                        uint64_t* pairs, int64_t cap) {
    try {
        return seam_pairs_impl(c, UpperIds32{upper32, upper_base}, lower, n, pairs, cap);
    } catch (const CCError& e) {
        g_err = e.msg;
        return -1;
    }
}

int64_t cc_seam_pairs_cubes32(cc_ctx* c, const uint32_t* upper_cubes, uint64_t upper_base, const uint64_t* lower,
                              int64_t Y, int64_t X, uint64_t* pairs, int64_t cap) {
    try {
        CC_REQUIRE(Y >= 1 && X >= 1 && Y * X < (1LL << 32), "bad plane shape");
        UpperCubes32 up{upper_cubes, upper_base, (u32)X, (u32)((X + 1) / 2)};
        return seam_pairs_impl(c, up, lower, Y * X, pairs, cap);
    } catch (const CCError& e) {
        g_err = e.msg;
        return -1;
    }
}

int cc_shard_top_cubes32(cc_ctx* c, uint32_t* cubes) {
    CC_TRY({
        CC_REQUIRE(c && cubes, "NULL argument");
        require_row_aligned(cubes, 4);
        HIP_OK(hipSetDevice(c->device));
        RunState& st = state(c);
        CC_REQUIRE(st.stage == 2, "phase order: call cc_shard_assign first");
        CC_REQUIRE(st.sum_v < (1ull << 28) - 2, "slab id range does not fit the 28-bit cube form");
        Geom& g = st.hg.g;
        for (int a = 1; a < 3; ++a)   // tile origins = block origins + multiples of TY / TX
            CC_REQUIRE(g.nb[a] == 1 || st.bs[a] % 2 == 0, "cube form needs even tile origins (even block_shape[1:])");
        hipStream_t s = cstream(c);
        const unsigned nlayer = (unsigned)((int64_t)g.nt[1] * g.nt[2]);
        launch(c, "k_top_cubes", [&] {
            k_top_cubes<<<nlayer, NTHREADS, 0, s>>>(g, c->faces.as<face_t>(), c->P.as<u32>(), c->KR.as<u64>(), cubes,
                                                     (u64)st.base, nullptr);
        });
    })
}

int cc_shard_top_plane32(cc_ctx* c, uint32_t* top32) {
    CC_TRY({
        CC_REQUIRE(c && top32, "NULL argument");
        require_row_aligned(top32, 4);
        HIP_OK(hipSetDevice(c->device));
        RunState& st = state(c);
        CC_REQUIRE(st.stage == 2, "phase order: call cc_shard_assign first");
        CC_REQUIRE(st.sum_v < 0xFFFFFFFEull, "slab id range does not fit the 32-bit plane form");
        Geom& g = st.hg.g;
        hipStream_t s = cstream(c);
        const unsigned nlayer = (unsigned)((int64_t)g.nt[1] * g.nt[2]);
        launch(c, "k_plane_labels", [&] {
            k_plane_labels<true, u32><<<nlayer, NTHREADS, 0, s>>>(g, c->faces.as<face_t>(), c->P.as<u32>(),
                                                                 c->KR.as<u64>(), top32, (u64)st.base);
        });
    })
}

int cc_shard_finish(cc_ctx* c, const uint64_t* pairs, int64_t n_pairs, uint64_t* labels, cc_result* res) {
    CC_TRY({
        CC_REQUIRE(c && labels && n_pairs >= 0 && (n_pairs == 0 || pairs), "bad arguments");
        HIP_OK(hipSetDevice(c->device));
        phase_map(c, pairs, n_pairs);
        phase_final(c, labels, res);
    })
}

}  // extern "C"

// ---------------------------------------------------------------------------------------------
// z-slab sharding, one-read-back schedule (distributed.py's default): the sums, the id base, the
// seam planes and pairs stay on the device between the collectives; cc_shard_dev_finish is the
// step's one host read-back.  Its status says whether every slab's optimistic assumptions held
// (the same answer on every rank: it is computed from the allgathered pair headers and sums);
// if not, the caller runs the host-synchronised schedule (cc_shard_begin ...) for this step.
// ---------------------------------------------------------------------------------------------
extern "C" {

int cc_shard_dev_ok(cc_ctx* c) { return c && fast_ok(c) ? 1 : 0; }

int cc_shard_dev_begin(cc_ctx* c, const float* in, const uint8_t* mask, const int64_t slab_shape[3],
                       const int64_t block_shape[3], double threshold, int mode, int64_t z_offset,
                       uint64_t* sum_dev) {
    CC_TRY({
        CC_REQUIRE(c && in && slab_shape && block_shape && sum_dev, "NULL argument");
        CC_REQUIRE(z_offset >= 0 && z_offset % block_shape[0] == 0,
                   "slab z offset must be a multiple of block_shape[0] (seams on block faces)");
        CC_REQUIRE(fast_ok(c), "the one-read-back schedule is off on this context (debug flags / options)");
        HIP_OK(hipSetDevice(c->device));
        phase_local(c, in, mask, slab_shape, block_shape, threshold, to_mode(mode), z_offset, false, true, sum_dev);
    })
}

int cc_shard_dev_assign(cc_ctx* c, const uint64_t* sums_dev, int rank, int world) {
    CC_TRY({
        CC_REQUIRE(c && sums_dev && rank >= 0 && rank < world, "bad arguments");
        HIP_OK(hipSetDevice(c->device));
        phase_rid_dev(c, sums_dev, rank);
    })
}

int cc_shard_dev_top_cubes(cc_ctx* c, uint32_t* cubes_dev) {
    CC_TRY({
        CC_REQUIRE(c && cubes_dev, "NULL argument");
        require_row_aligned(cubes_dev, 4);
        HIP_OK(hipSetDevice(c->device));
        RunState& st = state(c);
        CC_REQUIRE(st.stage == 2 && st.base_dev, "phase order: call cc_shard_dev_assign first");
        Geom& g = st.hg.g;
        for (int a = 1; a < 3; ++a)
            CC_REQUIRE(g.nb[a] == 1 || st.bs[a] % 2 == 0, "cube form needs even tile origins (even block_shape[1:])");
        hipStream_t s = cstream(c);
        const unsigned nlayer = (unsigned)((int64_t)g.nt[1] * g.nt[2]);
        launch(c, "k_top_cubes", [&] {
            k_top_cubes<<<nlayer, NTHREADS, 0, s>>>(g, c->faces.as<face_t>(), c->P.as<u32>(), c->KR.as<u64>(), cubes_dev,
                                                     0, c->scalars.as<u64>());
        });
    })
}

int cc_shard_dev_seam_pairs(cc_ctx* c, const uint32_t* upper_cubes_dev, const uint64_t* sums_dev, int rank,
                            uint64_t* hdr_pairs_dev, int64_t cap) {
    CC_TRY({
        CC_REQUIRE(c && sums_dev && hdr_pairs_dev && cap >= 0, "bad arguments");
        CC_REQUIRE(!upper_cubes_dev || rank > 0, "slab 0 has no slab below");
        HIP_OK(hipSetDevice(c->device));
        RunState& st = state(c);
        CC_REQUIRE(st.stage == 2 && st.base_dev, "phase order: call cc_shard_dev_assign first");
        Geom& g = st.hg.g;
        hipStream_t s = cstream(c);
        if (!upper_cubes_dev) {
            launch(c, "k_seam_hdr", [&] { k_seam_hdr<<<1, 64, 0, s>>>(c->scalars.as<u64>(), hdr_pairs_dev); });
            return 0;
        }
        for (int a = 1; a < 3; ++a)
            CC_REQUIRE(g.nb[a] == 1 || st.bs[a] % 2 == 0, "cube form needs even tile origins (even block_shape[1:])");
        // the seam pair hash set (see k_seam_cube_pairs) was cleared by this step's front clear (k_sample)
        const unsigned nlayer = (unsigned)((int64_t)g.nt[1] * g.nt[2]);
        launch(c, "k_seam_cube_pairs", [&] {
            k_seam_cube_pairs<<<nlayer, NTHREADS, 0, s>>>(g, c->faces.as<face_t>(), c->P.as<u32>(), c->KR.as<u64>(),
                                                           upper_cubes_dev, sums_dev, rank, hdr_pairs_dev, (u64)cap,
                                                           c->seam_hash.as<u64>(), (u32)(SEAM_SET - 1), c->scalars.as<u64>());
        });
        launch(c, "k_seam_hdr", [&] { k_seam_hdr<<<1, 64, 0, s>>>(c->scalars.as<u64>(), hdr_pairs_dev); });
    })
}

// all_dev: [world][cap + 1][2] (every slab's buffer of cc_shard_dev_seam_pairs, allgathered);
// status_host[4] (nullable): redo flags (RF_*: non-zero -> run this step host-synchronised), the
// largest pair count of a slab, the global n_labels, this slab's id base
int cc_shard_dev_finish(cc_ctx* c, const uint64_t* all_dev, int world, int64_t cap, const uint64_t* sums_dev,
                        uint64_t* labels_dev, cc_result* res, uint64_t* status_host) {
    CC_TRY({
        CC_REQUIRE(c && all_dev && sums_dev && labels_dev && world >= 1 && cap >= 0, "bad arguments");
        HIP_OK(hipSetDevice(c->device));
        SeamDev sd;
        sd.all = all_dev;
        sd.world = world;
        sd.cap = (uint64_t)cap;
        sd.sums = sums_dev;
        phase_final(c, labels_dev, res, &sd);
        RunState& st = state(c);
        if (status_host) {
            status_host[0] = st.redo;
            status_host[1] = st.n_pairs_max;
            status_host[2] = res ? res->n_labels : 0;
            status_host[3] = st.base;
        }
        // a slab with more roots than the capacity: room for them in the next step (the step is
        // redone host-synchronised, which counts them)
        if (st.redo & RF_ROOTS) c->root_cap = std::max<uint64_t>(c->root_cap, 2 * c->root_cap);
    })
}

}  // extern "C"

