// cc_ctx.hpp -- the host side shared by both translation units of libcc_mi355x.so (cc_lib.hip:
// the labelling path; cc_aux.hip: evaluation, relabelling, prefilter, watershed): the context,
// device memory (Arena / DevBuf), launches with optional event timing, synchronisation and
// read-backs, the C-ABI error convention (CC_TRY).  Two units, so that the labelling path's
// code object holds only its own kernels: the first launch from a code object loads all of its
// kernels (profiles/r04_cold_*).
#pragma once
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/cc_mi355x.h"
#include "cc_common.hpp"

using namespace cc;

inline thread_local std::string g_err;   // cc_last_error (one per thread, shared by both units)

#include "cc_host.hpp"

// integer from the environment (A/B knobs), read per call
static inline long env_int(const char* name, long dflt) {
    const char* e = std::getenv(name);
    return (e && *e) ? std::atol(e) : dflt;
}

// host time spent in device allocations (instrumentation of the cold, first-call cost: reported by
// cc_get_profile as the pseudo-kernel "host_alloc" -- count = hipMalloc calls, ms = their time)
inline std::atomic<int64_t> g_alloc_count{0}, g_alloc_ns{0};
// host synchronisations of the library's streams (reported as "host_sync": count, host ms waited)
inline std::atomic<int64_t> g_sync_count{0}, g_sync_ns{0};

// Device memory of every context comes from per-device chunks of at least 1 GiB, handed out
// first-fit in 256-B pieces.  In a fresh process each large hipMalloc / hipFree measured ~0.2 ms
// after a pageable upload (the one-shot job's first call made six of them, 1.0 ms, and as many
// frees at cc_destroy: profiles/r04_cold_*); a chunk pays that once.  Requests of LARGE bytes or
// more (volume-sized buffers of big inputs) get a chunk of their own, of their exact size, so the
// arena never holds gigabytes beside them.  A released piece is reused only once the work queued
// before its release has finished: release() records an event on the owner's stream (the
// context's stream, which its side stream has joined) and the piece waits in `pending` until the
// event completes -- no device-wide synchronisation, so RCCL collectives and other streams in
// flight are not waited for.  A piece released without an owner stream (the communicator's
// buffers) falls back to a device synchronisation.  A chunk is returned to HIP when its last piece
// is free and no pending piece refers to it.
struct Arena {
    struct Chunk {
        int dev;
        char* base;
        size_t size, live;
        std::map<size_t, size_t> free;   // offset -> bytes
    };
    struct Pending {
        Chunk* ch;
        size_t off, nb;
        hipEvent_t ev;
    };
    static constexpr size_t ALIGN = 256, MIN_CHUNK = size_t(1) << 30, GROW_CAP = size_t(2) << 30,
                            LARGE = size_t(256) << 20;
    std::mutex mu;
    std::vector<Chunk*> chunks;
    std::vector<Pending> pending;
    std::map<char*, std::pair<Chunk*, size_t>> owner;      // piece -> (chunk, bytes)

    void* take(Chunk* ch, std::map<size_t, size_t>::iterator it, size_t nb) {
        const size_t off = it->first, sz = it->second;
        ch->free.erase(it);
        if (sz > nb) ch->free[off + nb] = sz - nb;
        ch->live += 1;
        owner[ch->base + off] = {ch, nb};
        return ch->base + off;
    }
    // back into its chunk's free list (coalesced); the chunk is freed when nothing of it is live
    // or pending
    void put_back(Chunk* ch, size_t off, size_t nb) {
        auto nx = ch->free.lower_bound(off);
        if (nx != ch->free.end() && off + nb == nx->first) { nb += nx->second; nx = ch->free.erase(nx); }
        if (nx != ch->free.begin()) {
            auto pv = std::prev(nx);
            if (pv->first + pv->second == off) { off = pv->first; nb += pv->second; ch->free.erase(pv); }
        }
        ch->free[off] = nb;
        if (--ch->live == 0 && std::none_of(pending.begin(), pending.end(), [&](const Pending& q) { return q.ch == ch; })) {
            (void)hipFree(ch->base);
            chunks.erase(std::find(chunks.begin(), chunks.end(), ch));
            delete ch;
        }
    }
    // pending pieces whose event has completed (wait = true: all of them, waiting)
    void reap(bool wait) {
        for (size_t i = 0; i < pending.size();) {
            Pending q = pending[i];
            const hipError_t r = wait ? hipEventSynchronize(q.ev) : hipEventQuery(q.ev);
            if (r == hipErrorNotReady) { ++i; continue; }
            (void)hipGetLastError();
            (void)hipEventDestroy(q.ev);
            pending.erase(pending.begin() + i);
            q.ch->live += 1;              // put_back's accounting: the piece was counted live until now
            put_back(q.ch, q.off, q.nb);
        }
    }
    void* find_free(int dev, size_t nb, size_t* total) {
        for (Chunk* ch : chunks) {
            if (ch->dev != dev) continue;
            if (total) *total += ch->size;
            for (auto it = ch->free.begin(); it != ch->free.end(); ++it)
                if (it->second >= nb) return take(ch, it, nb);
        }
        return nullptr;
    }
    void* alloc(size_t need) {
        const size_t nb = (need + ALIGN - 1) & ~(ALIGN - 1);
        int dev = 0;
        HIP_OK(hipGetDevice(&dev));
        std::lock_guard<std::mutex> g(mu);
        reap(false);
        size_t total = 0;
        if (nb < LARGE) {
            if (void* p = find_free(dev, nb, &total)) return p;
            // pieces still in use by queued work: wait for them before growing the arena
            bool mine = false;
            for (const Pending& q : pending) mine |= q.ch->dev == dev;
            if (mine) {
                reap(true);
                if (void* p = find_free(dev, nb, nullptr)) return p;
            }
        }
        // a new chunk: a large request gets its own of its size; otherwise at least 1 GiB, growing
        // with what the device already holds (at most GROW_CAP beyond the request); the exact size
        // when that much is not available
        size_t cs = nb >= LARGE ? nb : std::max(nb, std::max(MIN_CHUNK, std::min(total, GROW_CAP)));
        cs = (cs + (size_t(2) << 20) - 1) & ~((size_t(2) << 20) - 1);
        char* base = nullptr;
        if (hipMalloc(&base, cs) != hipSuccess) {
            (void)hipGetLastError();
            reap(true);
            if (nb < LARGE)
                if (void* p = find_free(dev, nb, nullptr)) return p;
            cs = nb;
            HIP_OK(hipMalloc(&base, cs));
        }
        Chunk* ch = new Chunk{dev, base, cs, 0, {}};
        ch->free[0] = cs;
        chunks.push_back(ch);
        return take(ch, ch->free.begin(), nb);
    }
    // stream (nullable): the owner's stream; the piece is reusable once the work queued on it
    // so far has finished.  nullptr: a device synchronisation first (reusable at once).
    // the pieces whose event has completed back into the free lists (chunks freed when empty)
    void trim() {
        std::lock_guard<std::mutex> g(mu);
        reap(false);
    }
    void release(void* p, hipStream_t* stream = nullptr) {
        if (!p) return;
        hipEvent_t ev = nullptr;
        if (stream) {
            if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess || hipEventRecord(ev, *stream) != hipSuccess) {
                (void)hipGetLastError();
                if (ev) (void)hipEventDestroy(ev);
                ev = nullptr;
            }
        }
        if (!ev) (void)hipDeviceSynchronize();
        std::lock_guard<std::mutex> g(mu);
        auto o = owner.find((char*)p);
        if (o == owner.end()) {
            if (ev) (void)hipEventDestroy(ev);
            return;
        }
        Chunk* ch = o->second.first;
        const size_t off = (char*)p - ch->base, nb = o->second.second;
        owner.erase(o);
        if (ev) {
            ch->live -= 1;                 // counted again when reaped
            pending.push_back({ch, off, nb, ev});
        } else {
            put_back(ch, off, nb);
        }
    }
};
inline Arena g_arena;

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    hipStream_t* stream = nullptr;       // the owner's stream (deferred reuse on release), if bound
    template <class T>
    T* as() const { return (T*)p; }
    void ensure(size_t need) {
        if (need <= bytes && p) return;
        const auto t0 = std::chrono::steady_clock::now();
        const size_t before = g_arena.chunks.size();
        g_arena.release(p, stream);
        p = nullptr;
        bytes = 0;
        size_t nb = std::max<size_t>(need + need / 8, 256);
        p = g_arena.alloc(nb);
        bytes = nb;
        // host_alloc counts the allocations that reached HIP (new chunks)
        if (g_arena.chunks.size() > before) g_alloc_count += 1;
        const int64_t ns = std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
        g_alloc_ns += ns;
        static const bool log = std::getenv("CC_ALLOC_LOG") != nullptr;
        if (log) std::fprintf(stderr, "cc_alloc %zu B %.1f us chunks %zu\n", nb, ns * 1e-3, g_arena.chunks.size());
    }
    void release() {
        g_arena.release(p, stream);
        p = nullptr;
        bytes = 0;
    }
};

// pinned host memory for the pipeline's small read-backs: a copy into pageable memory went
// through the runtime's staging path (25-80 us of idle GPU per read in the C3 trace)
struct HostPin {
    void* p = nullptr;
    size_t bytes = 0;
    void* ensure(size_t n) {
        if (n > bytes) {
            if (p) HIP_OK(hipHostFree(p));
            p = nullptr;
            const size_t nb = std::max<size_t>(n, 64 << 10);
            HIP_OK(hipHostMalloc(&p, nb, hipHostMallocDefault));
            bytes = nb;
        }
        return p;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        bytes = 0;
    }
};

struct ProfEntry {
    int64_t count = 0;
    double ms = 0;
};

struct cc_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t side = nullptr;      // k_seams of finished front chunks, concurrent with the next chunk
    // workspace
    DevBuf tiles, bstat, bparam, bits, faces, count, rc, roff, rl, rcb, P, KR, FIN, keys, keys2, vals, vals2, seg,
        values, offsets, lut, cub_tmp, scalars, scalars2, counter, in_tmp, mask_tmp, out_tmp, pairs, pairs2,
        flags, map_ids, map_ids2, map_vals, map_par, big, pairsl, pc, ipairs, ipc, iovf, spec, mark, bflag,
        ev_main, ev_z, ev_seg, ev_gt, ev_flag, ev_part,   // evaluation (cc_eval.hip)
        rl_wg,                                            // relabel: per-workgroup id lists
        gs1, gs2, gs_tab,                                 // Gaussian prefilter temporaries (cc_prefilter.hip)
        mask_xmap,                                        // resized masks (cc_mask.hip)
        mlive,                                            // masked runs: blocks holding a mask voxel (k_mask_live)
        seam_hash,                                        // seam pair hash set (k_seam_pairs)
        ws_tab, ws_buf;                                   // seeded watershed (cc_watershed.hip)
    int64_t ev_cap = 0;      // entries per evaluation hash table of the last cc_evaluate
    int64_t rl_cap = 0;      // id-set slots of the last cc_relabel_consecutive
    // last run
    int64_t n_blocks = 0;
    uint64_t n_labels = 0;
    std::vector<uint64_t> h_values, h_offsets;
    std::vector<int32_t> h_tab;
    std::vector<int32_t> h_gs;   // Gaussian segment tables (cc_prefilter.hip AxSeg), alive until copied
    HostPin pin;             // small read-backs (see HostPin)
    bool lut_valid = false;
    // profiling
    int prof = 0;          // 0 off, 1 every launch, 2 the volume-sized kernels only (cc_set_profiling)
    int debug = 0;         // CC_DEBUG_* test hooks
    int front_chunks = 1;  // z-layer chunks of the speculative front (CC_FRONT_CHUNKS)
    int64_t quirk_jobs = 0;  // CC_OPT_EMPTY_JOB_QUIRK: emulate the reference's empty-job branch for max_jobs
    // one-read-back schedule (see run_pipeline): capacity of the root arrays sized before the count
    // is known (grown after a run that exceeded it), and whether the last volume of this geometry
    // needed the global-stitch fallback (then the host-synchronised schedule runs directly)
    bool ws_prenormalized = false;   // CC_OPT_WS_PRENORMALIZED
    uint64_t root_cap = 0;
    bool fast_big = false;
    std::vector<int32_t> fast_big_tab;
    // the sharded C entry (cc_comm.hip): geometry key of the last z-slab step whose status left
    // the one-read-back schedule for good (RF_BIG / RF_CUBES / RF_IOVF; 0 none)
    uint64_t shard_slow_key = 0;
    DevBuf status, hmap_keys, hmap_par;
    uint64_t hm_slots = 0;   // slots of the seam map (shards): cleared by the next front clear (k_sample)
    std::vector<std::pair<std::string, std::pair<hipEvent_t, hipEvent_t>>> pending;
    std::vector<hipEvent_t> event_pool;
    std::map<std::string, ProfEntry> prof_acc;
    void* run = nullptr;     // RunState of the current labelling run
};

// every device buffer of a context (bound to its stream at creation, released at destruction)
static inline std::vector<DevBuf*> ctx_bufs(cc_ctx* c) {
    return {&c->tiles, &c->bstat, &c->bparam, &c->bits, &c->faces, &c->count, &c->rc, &c->roff, &c->rl, &c->rcb, &c->P,
            &c->KR, &c->FIN, &c->keys, &c->keys2, &c->vals, &c->vals2, &c->seg, &c->values, &c->offsets, &c->lut,
            &c->cub_tmp, &c->scalars, &c->counter, &c->in_tmp, &c->mask_tmp, &c->out_tmp, &c->pairs, &c->pairs2,
            &c->scalars2, &c->flags, &c->map_ids, &c->map_ids2, &c->map_vals, &c->map_par, &c->big, &c->pairsl, &c->pc,
            &c->ipairs, &c->ipc, &c->iovf, &c->spec, &c->mark, &c->bflag, &c->ev_main, &c->ev_z, &c->ev_seg, &c->ev_gt,
            &c->ev_flag, &c->ev_part, &c->rl_wg, &c->gs1, &c->gs2, &c->gs_tab, &c->mask_xmap, &c->mlive, &c->seam_hash, &c->ws_tab,
            &c->ws_buf, &c->status, &c->hmap_keys, &c->hmap_par};
}

// the context's stream: the caller's (cc_set_stream), else the null stream -- which is torch's
// default stream too.  No stream of its own: creating one costs a hardware queue (10 ms in the
// C1 cold-call trace, profiles/r03_c1_trace_*), paid by every one-shot job.
static hipStream_t cstream(cc_ctx* c) { return c->stream; }
// the side stream (k_seams of finished front chunks), created on first use
static hipStream_t side_stream(cc_ctx* c) {
    if (!c->side) HIP_OK(hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
    return c->side;
}

// ------------------------------------------------------------------------------------------
// helpers
// ------------------------------------------------------------------------------------------
static hipEvent_t pool_event(cc_ctx* c) {
    if (!c->event_pool.empty()) {
        hipEvent_t e = c->event_pool.back();
        c->event_pool.pop_back();
        return e;
    }
    hipEvent_t e;
    HIP_OK(hipEventCreate(&e));
    return e;
}

template <class F>
static void launch_on(cc_ctx* c, hipStream_t s, const char* name, F&& f) {
    hipEvent_t a = nullptr, b = nullptr;
    const bool timed = c->prof == 1 || (c->prof == 2 && (!std::strcmp(name, "k_spec") || !std::strcmp(name, "k_pass2")));
    if (timed) {
        a = pool_event(c);
        b = pool_event(c);
        HIP_OK(hipEventRecord(a, s));
    }
    f();
    HIP_OK(hipGetLastError());
    if (timed) {
        HIP_OK(hipEventRecord(b, s));
        c->pending.push_back({name, {a, b}});
    }
}

template <class F>
static void launch(cc_ctx* c, const char* name, F&& f) { launch_on(c, cstream(c), name, static_cast<F&&>(f)); }

// stream `waiter` waits for the work enqueued so far on `from`
static void stream_wait(cc_ctx* c, hipStream_t from, hipStream_t waiter) {
    hipEvent_t e;
    HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIP_OK(hipEventRecord(e, from));
    HIP_OK(hipStreamWaitEvent(waiter, e, 0));
    HIP_OK(hipEventDestroy(e));
}

static void resolve_profile(cc_ctx* c) {
    for (auto& pe : c->pending) {
        float ms = 0;
        HIP_OK(hipEventElapsedTime(&ms, pe.second.first, pe.second.second));
        auto& acc = c->prof_acc[pe.first];
        acc.count += 1;
        acc.ms += ms;
        c->event_pool.push_back(pe.second.first);
        c->event_pool.push_back(pe.second.second);
    }
    c->pending.clear();
}

// While the sharded C entry runs (cc_comm.hip), host synchronisations go through its bounded
// wait: it polls the stream with a deadline and the communicator's asynchronous error, so a peer
// that failed between collectives ends this rank's wait with an error instead of a hang.
struct SyncHook {
    void (*wait)(void* arg, hipStream_t s);
    void* arg;
};
static thread_local SyncHook* g_sync_hook = nullptr;

static void stream_sync(hipStream_t st) {
    const auto t0 = std::chrono::steady_clock::now();
    if (g_sync_hook) g_sync_hook->wait(g_sync_hook->arg, st);
    else HIP_OK(hipStreamSynchronize(st));
    g_sync_count += 1;
    g_sync_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
}

static void sync(cc_ctx* c) {
    stream_sync(cstream(c));
    if (c->prof) resolve_profile(c);
}

// read-backs through the pinned buffer: enqueue (device src, bytes) pieces at increasing offsets,
// one synchronisation, then copy out on the host.  Nothing else may use c->pin meanwhile.
struct Readback {
    cc_ctx* c;
    size_t off = 0;
    std::vector<std::pair<void*, std::pair<size_t, size_t>>> outs;   // (host dst, (offset, bytes))
    Readback(cc_ctx* c_, size_t total) : c(c_) { c->pin.ensure(total); }
    void add(void* dst, const void* src, size_t bytes) {
        off = (off + 15) & ~size_t(15);
        if (bytes) HIP_OK(hipMemcpyAsync((char*)c->pin.p + off, src, bytes, hipMemcpyDeviceToHost, cstream(c)));
        outs.push_back({dst, {off, bytes}});
        off += bytes;
    }
    // resolve = false: the side stream may still run timed kernels (the k_fix count is read
    // while k_seams runs), so the stream is synchronised without resolving the profile events
    void wait(bool resolve = true) {
        if (resolve) sync(c);
        else stream_sync(cstream(c));
        for (auto& o : outs) if (o.second.second) std::memcpy(o.first, (char*)c->pin.p + o.second.first, o.second.second);
    }
};

// 1-D grid; element kernels index one element per thread, so n must stay below 2^32 threads
// (volume-sized kernels use CC_FOR with the grid capped by grid_stride()).
static inline unsigned grid1d(int64_t n, int bs = 256) {
    CC_REQUIRE(n < (1LL << 32) - bs, "1-D launch larger than 2^32 threads");
    return (unsigned)std::max<int64_t>(1, (n + bs - 1) / bs);
}
static inline unsigned grid_stride(int64_t n, int bs = 256) { return (unsigned)std::min<int64_t>(1 << 20, std::max<int64_t>(1, (n + bs - 1) / bs)); }

static void upload_geom(cc_ctx* c, HostGeom& hg) {
    // the tables of the last upload are still on the device when the geometry repeats (the
    // common case: one volume shape per context); otherwise upload (h_tab stays alive in the ctx
    // until the stream has consumed it)
    const size_t bytes = hg.tab.size() * sizeof(int32_t);
    const size_t cap_before = c->tiles.bytes;      // ensure() only reallocates to a larger size
    c->tiles.ensure(bytes);
    if (!(c->tiles.bytes == cap_before && c->h_tab == hg.tab)) {
        c->h_tab = hg.tab;
        HIP_OK(hipMemcpyAsync(c->tiles.p, c->h_tab.data(), bytes, hipMemcpyHostToDevice, cstream(c)));
    }
    bind_geom_tables(hg, c->tiles.as<int32_t>());
}

static int to_mode(int mode) {
    CC_REQUIRE(mode >= 0 && mode <= 2, "mode must be 0 (greater), 1 (less) or 2 (equal)");
    return mode;
}

// state of the context's current labelling run (cc_lib.hip's phases; the normalisation steps of
// cc_aux.hip keep their geometry here too)
struct RunState {
    HostGeom hg;
    float thr = 0.f;
    int mode = 0;
    int64_t nr = 0;            // block-local roots
    uint64_t sum_v = 0;        // sum of block values of this volume / slab
    uint64_t base = 0;         // global id base of this slab
    int64_t n_map = 0;         // seam mapping size
    bool local_only = false;
    bool masked = false;       // a mask was given (k_pass2's tile order)
    int64_t bs[3] = {0, 0, 0};  // block_shape
    uint64_t n_fix = 0;        // tiles relabelled by k_fix
    bool identity_lut = false; // the empty-job emulation dropped every block-face merge
    int stage = 0;             // 1 local done, 2 rid done, 3 final done
    bool rid0 = false;         // k_emit_roots already wrote the roots' ids for base 0
    bool sum_known = false;    // sum_v already read back (phase_local's fast path)
    bool any_iovf = true;      // some tile's block-face pair list overflowed (or not read back)
    bool fast = false;         // the one-read-back schedule: counts stay on the device
    bool base_dev = false;     // ids of this slab stay base 0; kernels add the allgathered sums below it
    uint64_t redo = 0;         // RF_* flags read back by phase_final (fast schedule): run again synchronised
    uint64_t n_pairs_max = 0;  // largest seam-pair count of a slab (shards of the fast schedule)
    const uint64_t* sums = nullptr;   // the allgathered sums (shards of the fast schedule)
    int rank = 0;
};

static RunState& state(cc_ctx* c) {
    if (!c->run) c->run = new RunState();
    return *(RunState*)c->run;
}

// ------------------------------------------------------------------------------------------
// C ABI error convention: 0 ok, -1 CCError (message in cc_last_error), -2 other exceptions
// ------------------------------------------------------------------------------------------
#define CC_TRY(...)                                                                            \
    try {                                                                                      \
        __VA_ARGS__;                                                                           \
        return 0;                                                                              \
    } catch (const CCError& e) {                                                               \
        g_err = e.msg;                                                                         \
        return -1;                                                                             \
    } catch (const std::exception& e) {                                                        \
        g_err = e.what();                                                                      \
        return -2;                                                                             \
    }

