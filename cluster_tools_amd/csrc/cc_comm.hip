// cc_comm.hip -- z-slab sharding with RCCL inside the library (included at the end of cc_lib.hip,
// same translation unit): a C caller shards a volume over the GPUs of a node without torch.
//
// The reference runs block_components / block_faces / write as jobs of a process pool
// (/root/reference/cluster_tools/cluster_tasks.py:529-551) and exchanges offsets and face
// assignments through files; here each rank owns a z-slab of the volume on its GPU and the three
// exchanges of the schedule run as RCCL collectives on the context's stream:
//   one-read-back schedule (distributed.py's default, cc_shard_dev_*): allgather of the slabs'
//     sums of block values (8 B per rank), the top seam plane in the cube form to rank + 1
//     (point-to-point over one xGMI link), allgather of the fixed-capacity seam-pair buffers; the
//     step's one host read-back is the status of cc_shard_dev_finish;
//   host-synchronised schedule (the redo path, uint64 seam planes: any id range, any block
//     shape): counts read back, padded allgather of the seam pairs, cc_shard_finish.
//
// Every call starts with an AGREEMENT: each rank checks its own arguments, then the ranks
// allgather a 16-word header (ok flag, proposed schedule, global shape, block shape, slab bounds,
// mode, threshold, mask) on the communicator's side stream while the rank's front
// (cc_shard_dev_begin) already runs on the main stream, so the round trip costs no step time.
// A bad argument on any rank, or ranks that disagree on the volume, or slabs that do not tile it
// in rank order, make EVERY rank return an error before any data-path collective is queued; the
// communicator stays usable.  The schedule is the minimum of the proposals (cube form possible
// for these block shapes, cc_shard_dev_ok, no sticky fallback of this geometry on the context).
// A step whose status carries redo flags is relabelled synchronised; RF_PAIRS raises the pair
// capacity, RF_BIG / RF_CUBES / RF_IOVF keep this geometry synchronised on the context.
//
// Errors after the agreement (a failed collective, a kernel launch error, an allocation failure
// on one rank) ABORT the communicator (ncclCommAbort): RCCL's abort flag ends the peers' pending
// collectives, every host wait of the call is bounded (CC_COMM_TIMEOUT seconds, default 300) and
// polls ncclCommGetAsyncError, so the peers return an error too instead of hanging.  An aborted
// communicator refuses further calls; cc_comm_destroy frees it.
//
// RCCL is opened at the first cc_comm call (dlopen): the library itself needs no RCCL to load,
// and inside a process that already holds one (torch's), that copy is reused.  CC_RCCL_PATH names
// another library with the same entry points (the tests' shared-memory stand-in,
// tests/fake_rccl, which lets 2-3 ranks share the one GPU of a test box).
#include <dlfcn.h>
#include <unistd.h>

#include <rccl/rccl.h>

namespace {

struct RcclApi {
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
    // optional: without them an error after the agreement leaks the communicator (no abort) and
    // the bounded waits rely on the deadline alone
    ncclResult_t (*abort)(ncclComm_t) = nullptr;
    ncclResult_t (*async_error)(ncclComm_t, ncclResult_t*) = nullptr;
};

const RcclApi& rccl() {
    static RcclApi api;
    static std::once_flag once;
    static std::string err;
    std::call_once(once, [] {
        void* h = nullptr;
        if (const char* p = std::getenv("CC_RCCL_PATH"); p && *p) {
            h = dlopen(p, RTLD_NOW | RTLD_LOCAL);
            if (!h) { err = std::string("CC_RCCL_PATH: ") + dlerror(); return; }
        }
        // a copy already in the process (torch's) first, then the system one
        for (const char* name : {"librccl.so", "librccl.so.1"})
            if (!h) h = dlopen(name, RTLD_NOW | RTLD_NOLOAD);
        for (const char* name : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1"})
            if (!h) h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
        if (!h) { err = std::string("RCCL not found: ") + dlerror(); return; }
        auto sym = [&](const char* n) {
            void* f = dlsym(h, n);
            if (!f && err.empty()) err = std::string("RCCL symbol missing: ") + n;
            return f;
        };
        api.get_unique_id = (decltype(api.get_unique_id))sym("ncclGetUniqueId");
        api.init_rank = (decltype(api.init_rank))sym("ncclCommInitRank");
        api.destroy = (decltype(api.destroy))sym("ncclCommDestroy");
        api.all_gather = (decltype(api.all_gather))sym("ncclAllGather");
        api.send = (decltype(api.send))sym("ncclSend");
        api.recv = (decltype(api.recv))sym("ncclRecv");
        api.group_start = (decltype(api.group_start))sym("ncclGroupStart");
        api.group_end = (decltype(api.group_end))sym("ncclGroupEnd");
        api.error_string = (decltype(api.error_string))sym("ncclGetErrorString");
        api.abort = (decltype(api.abort))dlsym(h, "ncclCommAbort");
        api.async_error = (decltype(api.async_error))dlsym(h, "ncclCommGetAsyncError");
        if (!err.empty()) api.get_unique_id = nullptr;
    });
    CC_REQUIRE(api.get_unique_id != nullptr, err.empty() ? std::string("RCCL unavailable") : err);
    return api;
}

#define RCCL_OK(x)                                                                                 \
    do {                                                                                           \
        const ncclResult_t r_ = (x);                                                               \
        if (r_ != ncclSuccess) throw CCError{std::string("RCCL: ") + #x + ": " + rccl().error_string(r_)}; \
    } while (0)

constexpr int HDR_WORDS = 16;   // the agreement header (see agree())

}  // namespace

struct cc_comm {
    ncclComm_t comm = nullptr;
    int world = 1, rank = 0, device = 0;
    hipStream_t stream = nullptr;          // used when the context has no stream of its own
    hipStream_t astream = nullptr;         // the agreement's allgather (overlaps the front)
    hipEvent_t fence = nullptr, wait_ev = nullptr;
    int64_t pair_cap = 2048;               // seam pairs per slab of the one-read-back buffers
    double timeout_s = 300;                // bound of every host wait inside a call
    bool broken = false;                   // aborted: every later call fails fast
    std::string why;
    int64_t last_schedule = -1;            // 1 one-read-back, 0 synchronised (cc_comm_info)
    uint64_t last_redo = 0;                // RF_* flags of the last one-read-back attempt
    int64_t calls = 0;
    int fail_at = 0, n_coll = 0;           // CC_COMM_FAIL_AT: injected error after that collective (tests)
    DevBuf agree, sum, sums, top, upper, hdr, all, h8, bottom, top64, upper64, pairs, pad, allp;
};

static uint64_t next_pow2_u64(uint64_t n) {
    uint64_t p = 1;
    while (p < n) p <<= 1;
    return p;
}

// the bounded host wait installed as g_sync_hook for the duration of a call (cc_ctx.hpp)
static void comm_wait(void* arg, hipStream_t s) {
    cc_comm* m = (cc_comm*)arg;
    HIP_OK(hipEventRecord(m->wait_ev, s));
    const auto t0 = std::chrono::steady_clock::now();
    for (int spin = 0;; ++spin) {
        const hipError_t e = hipEventQuery(m->wait_ev);
        if (e == hipSuccess) return;
        if (e != hipErrorNotReady) HIP_OK(e);
        if ((spin & 63) == 63) {
            if (m->comm && rccl().async_error) {
                ncclResult_t ae = ncclSuccess;
                if (rccl().async_error(m->comm, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress)
                    throw CCError{std::string("RCCL asynchronous error: ") + rccl().error_string(ae)};
            }
            const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            if (el > m->timeout_s)
                throw CCError{"timed out after " + std::to_string((int)m->timeout_s) +
                              " s waiting for the z-slab exchange (a peer failed or stopped)"};
        }
        // busy-poll for the first 50 ms (a step's waits are shorter: no wake-up latency), then
        // yield the core between polls
        if (spin > 4096 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(50)) usleep(50);
    }
}

// one call's stream set-up: the context's stream (the caller's, cc_set_stream), else the
// communicator's own, ordered after the work already queued on the null stream (torch's default
// stream) and with the null stream ordered after the call; host waits bounded (comm_wait)
struct ShardCall {
    cc_ctx* c;
    cc_comm* m;
    hipStream_t saved;
    bool own;
    SyncHook hook;
    SyncHook* prev;
    ShardCall(cc_ctx* c_, cc_comm* m_) : c(c_), m(m_), saved(c_->stream), own(!c_->stream), hook{comm_wait, m_}, prev(g_sync_hook) {
        if (own) {
            HIP_OK(hipEventRecord(m->fence, nullptr));
            HIP_OK(hipStreamWaitEvent(m->stream, m->fence, 0));
            c->stream = m->stream;
        }
        g_sync_hook = &hook;
        m->n_coll = 0;
        m->fail_at = (int)env_int("CC_COMM_FAIL_AT", 0);
    }
    ~ShardCall() {
        g_sync_hook = prev;
        if (own && !m->broken && hipEventRecord(m->fence, m->stream) == hipSuccess)
            (void)hipStreamWaitEvent(nullptr, m->fence, 0);
        c->stream = saved;
    }
};

// after each collective: the tests' injected failure (CC_COMM_FAIL_AT=k: this rank fails after
// its k-th collective of the call, as a rank-local error would)
static void collective_done(cc_comm* m) {
    if (m->fail_at && ++m->n_coll == m->fail_at) throw CCError{"injected failure after collective " + std::to_string(m->fail_at)};
}

// allgather of one uint64 per rank through device memory (host values, one synchronisation)
static std::vector<uint64_t> allgather_u64(cc_ctx* c, cc_comm* m, uint64_t v) {
    hipStream_t s = cstream(c);
    m->h8.ensure((1 + (size_t)m->world) * sizeof(u64));
    u64* d = m->h8.as<u64>();
    HIP_OK(hipMemcpyAsync(d, &v, sizeof(u64), hipMemcpyHostToDevice, s));
    RCCL_OK(rccl().all_gather(d, d + 1, 1, ncclUint64, m->comm, s));
    collective_done(m);
    std::vector<uint64_t> out(m->world);
    HIP_OK(hipMemcpyAsync(out.data(), d + 1, m->world * sizeof(u64), hipMemcpyDeviceToHost, s));
    stream_sync(s);
    return out;
}

// to rank + 1 / from rank - 1 (either may be absent), one group
static void shift_up(cc_comm* m, hipStream_t s, const void* send, void* recv, size_t count, ncclDataType_t dt) {
    const bool tx = send && m->rank + 1 < m->world, rx = recv && m->rank > 0;
    if (!tx && !rx) return;
    RCCL_OK(rccl().group_start());
    if (tx) RCCL_OK(rccl().send(send, count, dt, m->rank + 1, m->comm, s));
    if (rx) RCCL_OK(rccl().recv(recv, count, dt, m->rank - 1, m->comm, s));
    RCCL_OK(rccl().group_end());
    collective_done(m);
}

static void check_rc(int rc) {
    if (rc < 0) throw CCError{g_err};
}

// abort the communicator after an error that may have left peers inside a collective
static void abort_comm(cc_comm* m, const std::string& why) {
    if (m->broken) return;
    m->broken = true;
    m->why = why;
    if (m->comm && rccl().abort) {
        (void)rccl().abort(m->comm);
        m->comm = nullptr;                 // freed by the abort
    }
}

static uint64_t fnv(const uint64_t* w, int n) {
    uint64_t h = 1469598103934665603ull;
    for (int i = 0; i < n; ++i) {
        h ^= w[i];
        h *= 1099511628211ull;
    }
    return h ? h : 1;
}

// the agreement: every rank's header allgathered on the side stream; the host waits (bounded)
enum { H_OK, H_FAST, H_Z, H_Y, H_X, H_B0, H_B1, H_B2, H_Z0, H_DEPTH, H_MODE, H_THR, H_MASK, H_WORLD };
static std::vector<uint64_t> agree(cc_comm* m, const uint64_t* hdr) {
    const size_t w = (size_t)m->world;
    m->agree.ensure((1 + w) * HDR_WORDS * sizeof(u64));
    u64* d = m->agree.as<u64>();
    std::vector<uint64_t> all(w * HDR_WORDS);
    HIP_OK(hipMemcpyAsync(d, hdr, HDR_WORDS * sizeof(u64), hipMemcpyHostToDevice, m->astream));
    RCCL_OK(rccl().all_gather(d, d + HDR_WORDS, HDR_WORDS, ncclUint64, m->comm, m->astream));
    collective_done(m);
    HIP_OK(hipMemcpyAsync(all.data(), d + HDR_WORDS, w * HDR_WORDS * sizeof(u64), hipMemcpyDeviceToHost, m->astream));
    stream_sync(m->astream);
    return all;
}

// the same verdict on every rank (computed from the same allgathered headers)
static void check_agreement(const std::vector<uint64_t>& all, int world) {
    auto at = [&](int r, int k) { return all[(size_t)r * HDR_WORDS + k]; };
    for (int r = 0; r < world; ++r)
        if (!at(r, H_OK)) throw CCError{"rank " + std::to_string(r) + " rejected its arguments (its own error says why); no rank ran the step"};
    for (int r = 1; r < world; ++r)
        for (int k : {H_Z, H_Y, H_X, H_B0, H_B1, H_B2, H_MODE, H_THR, H_MASK, H_WORLD})
            if (at(r, k) != at(0, k))
                throw CCError{"ranks 0 and " + std::to_string(r) + " disagree on the volume (shape, block_shape, mode, threshold, mask)"};
    uint64_t z = 0;
    for (int r = 0; r < world; ++r) {
        if (at(r, H_Z0) != z)
            throw CCError{"the slabs do not tile the volume in rank order: rank " + std::to_string(r) + " starts at z=" +
                          std::to_string(at(r, H_Z0)) + ", expected " + std::to_string(z)};
        z += at(r, H_DEPTH);
    }
    if (z != at(0, H_Z)) throw CCError{"the slabs end at z=" + std::to_string(z) + ", the volume at " + std::to_string(at(0, H_Z))};
}

extern "C" {

int cc_comm_unique_id(void* id_out, int64_t cap) {
    CC_TRY({
        CC_REQUIRE(id_out && cap >= (int64_t)sizeof(ncclUniqueId), "id buffer smaller than 128 bytes");
        ncclUniqueId id;
        RCCL_OK(rccl().get_unique_id(&id));
        std::memcpy(id_out, &id, sizeof(id));
    })
}

int cc_comm_create(const void* id, int world, int rank, int device, cc_comm** out) {
    CC_TRY({
        CC_REQUIRE(id && out && world >= 1 && rank >= 0 && rank < world, "bad arguments");
        int n = 0;
        HIP_OK(hipGetDeviceCount(&n));
        CC_REQUIRE(device >= 0 && device < n, "no such HIP device");
        HIP_OK(hipSetDevice(device));
        cc_comm* m = new cc_comm();
        m->world = world;
        m->rank = rank;
        m->device = device;
        m->pair_cap = std::max<int64_t>(1, env_int("CC_SHARD_PAIR_CAP", 2048));
        if (const char* e = std::getenv("CC_COMM_TIMEOUT"); e && *e) m->timeout_s = std::max(1.0, std::atof(e));
        ncclUniqueId uid;
        std::memcpy(&uid, id, sizeof(uid));
        try {
            HIP_OK(hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking));
            HIP_OK(hipStreamCreateWithFlags(&m->astream, hipStreamNonBlocking));
            for (hipEvent_t* e : {&m->fence, &m->wait_ev}) HIP_OK(hipEventCreateWithFlags(e, hipEventDisableTiming));
            RCCL_OK(rccl().init_rank(&m->comm, world, uid, rank));
        } catch (...) {
            for (hipStream_t st : {m->stream, m->astream}) if (st) (void)hipStreamDestroy(st);
            for (hipEvent_t e : {m->fence, m->wait_ev}) if (e) (void)hipEventDestroy(e);
            delete m;
            throw;
        }
        *out = m;
    })
}

// out[0..7]: world, rank, last schedule (1 one-read-back, 0 synchronised, -1 none yet), RF_* flags
// of the last one-read-back attempt, seam-pair capacity, aborted, calls, 0
int cc_comm_info(const cc_comm* m, int64_t* out) {
    CC_TRY({
        CC_REQUIRE(m && out, "NULL argument");
        const int64_t v[8] = {m->world, m->rank, m->last_schedule, (int64_t)m->last_redo, m->pair_cap, m->broken ? 1 : 0, m->calls, 0};
        std::memcpy(out, v, sizeof(v));
    })
}

void cc_comm_destroy(cc_comm* m) {
    if (!m) return;
    (void)hipSetDevice(m->device);
    // an aborted communicator's collectives have ended (RCCL's abort flag); its stream drains
    for (hipStream_t st : {m->stream, m->astream}) if (st) (void)hipStreamSynchronize(st);
    DevBuf* bufs[] = {&m->agree, &m->sum, &m->sums, &m->top, &m->upper, &m->hdr, &m->all, &m->h8, &m->bottom, &m->top64,
                      &m->upper64, &m->pairs, &m->pad, &m->allp};
    for (DevBuf* b : bufs) b->release();
    if (m->comm) (void)rccl().destroy(m->comm);
    for (hipStream_t st : {m->stream, m->astream}) if (st) (void)hipStreamDestroy(st);
    for (hipEvent_t e : {m->fence, m->wait_ev}) if (e) (void)hipEventDestroy(e);
    delete m;
}

int cc_label_volume_sharded(cc_ctx* c, cc_comm* m, const float* slab_dev, const uint8_t* mask_dev,
                            const int64_t global_shape[3], int64_t z_offset, int64_t slab_depth,
                            const int64_t block_shape[3], double threshold, int mode, uint64_t* labels_dev,
                            cc_result* res) {
    CC_TRY({
        CC_REQUIRE(c && m, "NULL context or communicator");
        CC_REQUIRE(!m->broken, "the communicator was aborted by an earlier error (" + m->why + "); destroy it");
        CC_REQUIRE(c->device == m->device, "context and communicator on different devices");
        HIP_OK(hipSetDevice(c->device));
        ShardCall call(c, m);
        m->calls += 1;
        hipStream_t s = cstream(c);
        const int world = m->world, rank = m->rank;
        // 1. this rank's own checks; a rank that fails them still takes part in the agreement
        std::string local_err;
        bool cubes_ok = false;
        try {
            CC_REQUIRE(slab_dev && global_shape && block_shape && labels_dev && res, "NULL argument");
            for (int a = 0; a < 3; ++a) CC_REQUIRE(global_shape[a] >= 1 && block_shape[a] >= 1, "bad shape / block_shape");
            CC_REQUIRE(slab_depth >= 1 && z_offset >= 0 && z_offset + slab_depth <= global_shape[0], "bad slab");
            CC_REQUIRE(z_offset % block_shape[0] == 0 && (slab_depth % block_shape[0] == 0 || z_offset + slab_depth == global_shape[0]),
                       "slabs must start and end on block faces");
            (void)to_mode(mode);
            require_row_aligned(slab_dev, global_shape[2] * 4);
            require_row_aligned(mask_dev, global_shape[2]);
            require_row_aligned(labels_dev, global_shape[2] * 8);
            const int64_t nby = (global_shape[1] + block_shape[1] - 1) / block_shape[1];
            const int64_t nbx = (global_shape[2] + block_shape[2] - 1) / block_shape[2];
            cubes_ok = (nby == 1 || block_shape[1] % 2 == 0) && (nbx == 1 || block_shape[2] % 2 == 0);
        } catch (const CCError& e) {
            local_err = e.msg;
        }
        uint64_t hdr[HDR_WORDS] = {};
        float thr = (float)threshold;
        hdr[H_OK] = local_err.empty();
        if (local_err.empty()) {
            const uint64_t geo[8] = {(u64)global_shape[0], (u64)global_shape[1], (u64)global_shape[2], (u64)block_shape[0],
                                     (u64)block_shape[1], (u64)block_shape[2], (u64)z_offset, (u64)slab_depth};
            const bool sticky = c->shard_slow_key && c->shard_slow_key == fnv(geo, 8);
            hdr[H_FAST] = cubes_ok && fast_ok(c) && !sticky;
            std::memcpy(&hdr[H_Z], geo, sizeof(geo));
            hdr[H_MODE] = (u64)mode;
            std::memcpy(&hdr[H_THR], &thr, sizeof(thr));
            hdr[H_MASK] = mask_dev != nullptr;
        }
        hdr[H_WORLD] = (u64)world;
        const int64_t slab[3] = {slab_depth, local_err.empty() ? global_shape[1] : 1, local_err.empty() ? global_shape[2] : 1};
        const int64_t Y = slab[1], X = slab[2];
        const int64_t ncube = ((Y + 1) / 2) * ((X + 1) / 2);
        // 2. the front of the one-read-back schedule, speculatively, while the ranks agree
        if (hdr[H_FAST]) {
            try {
                const int64_t cap = m->pair_cap;
                m->sum.ensure(sizeof(u64));
                m->sums.ensure(world * sizeof(u64));
                m->top.ensure(ncube * sizeof(u32));
                m->upper.ensure(ncube * sizeof(u32));
                m->hdr.ensure((cap + 1) * 2 * sizeof(u64));
                m->all.ensure((size_t)world * (cap + 1) * 2 * sizeof(u64));
                check_rc(cc_shard_dev_begin(c, slab_dev, mask_dev, slab, block_shape, threshold, mode, z_offset, m->sum.as<u64>()));
            } catch (const CCError& e) {
                local_err = e.msg;
                hdr[H_OK] = hdr[H_FAST] = 0;
            }
        }
        std::vector<uint64_t> all;
        try {
            all = agree(m, hdr);
        } catch (const CCError& e) {
            abort_comm(m, e.msg);
            throw;
        }
        if (!local_err.empty()) throw CCError{local_err};
        check_agreement(all, world);
        bool fast = true;
        for (int r = 0; r < world; ++r) fast = fast && all[(size_t)r * HDR_WORDS + H_FAST];
        const uint64_t geo[8] = {(u64)global_shape[0], (u64)Y, (u64)X, (u64)block_shape[0], (u64)block_shape[1],
                                 (u64)block_shape[2], (u64)z_offset, (u64)slab_depth};
        // 3. the schedule; an error from here on may leave peers inside a collective: abort
        try {
            if (fast) {
                const int64_t cap = m->pair_cap;
                u64* sums = m->sums.as<u64>();
                RCCL_OK(rccl().all_gather(m->sum.p, sums, 1, ncclUint64, m->comm, s));
                collective_done(m);
                check_rc(cc_shard_dev_assign(c, sums, rank, world));
                if (rank + 1 < world) check_rc(cc_shard_dev_top_cubes(c, m->top.as<u32>()));
                shift_up(m, s, m->top.p, m->upper.p, (size_t)ncube, ncclUint32);
                check_rc(cc_shard_dev_seam_pairs(c, rank > 0 ? m->upper.as<u32>() : nullptr, sums, rank, m->hdr.as<u64>(), cap));
                RCCL_OK(rccl().all_gather(m->hdr.p, m->all.p, (size_t)(cap + 1) * 2, ncclUint64, m->comm, s));
                collective_done(m);
                uint64_t status[4] = {0, 0, 0, 0};
                check_rc(cc_shard_dev_finish(c, m->all.as<u64>(), world, cap, sums, labels_dev, res, status));
                m->last_redo = status[0];
                m->last_schedule = 1;
                if (!status[0]) return 0;
                // every rank reads the same flags (computed from the allgathered headers and sums)
                if (status[0] & RF_PAIRS) m->pair_cap = (int64_t)next_pow2_u64(2 * status[1]);
                if (status[0] & (RF_BIG | RF_CUBES | RF_IOVF)) c->shard_slow_key = fnv(geo, 8);
            }
            // (a speculative front of a step another rank sent synchronised is dropped:
            // cc_shard_begin runs the front again and every output is rewritten)
            m->last_schedule = 0;
            // host-synchronised schedule with uint64 seam planes
            uint64_t sum_v = 0;
            check_rc(cc_shard_begin(c, slab_dev, mask_dev, slab, block_shape, threshold, mode, z_offset, &sum_v));
            const auto sums = allgather_u64(c, m, sum_v);
            uint64_t base = 0, total = 0;
            for (int r = 0; r < world; ++r) {
                if (r < rank) base += sums[r];
                total += sums[r];
            }
            check_rc(cc_shard_assign(c, base));
            const int64_t n = Y * X;
            if (rank > 0) { m->bottom.ensure(n * sizeof(u64)); m->upper64.ensure(n * sizeof(u64)); m->pairs.ensure(2 * n * sizeof(u64)); }
            if (rank + 1 < world) m->top64.ensure(n * sizeof(u64));
            check_rc(cc_shard_planes(c, rank > 0 ? m->bottom.as<u64>() : nullptr, rank + 1 < world ? m->top64.as<u64>() : nullptr));
            shift_up(m, s, m->top64.p, m->upper64.p, (size_t)n, ncclUint64);
            int64_t np = 0;
            if (rank > 0) {
                np = cc_seam_pairs(c, m->upper64.as<u64>(), m->bottom.as<u64>(), n, m->pairs.as<u64>(), n);
                check_rc((int)std::min<int64_t>(np, 0));
            }
            const auto counts = allgather_u64(c, m, (uint64_t)np);
            uint64_t mx = 0;
            for (uint64_t v : counts) mx = std::max(mx, v);
            const u64* allp = nullptr;
            if (mx) {
                // RCCL has no allgatherv: every rank's pairs padded with (0, 0) to the largest count
                m->pad.ensure(mx * 2 * sizeof(u64));
                m->allp.ensure((size_t)world * mx * 2 * sizeof(u64));
                HIP_OK(hipMemsetAsync(m->pad.p, 0, mx * 2 * sizeof(u64), s));
                if (np) HIP_OK(hipMemcpyAsync(m->pad.p, m->pairs.p, np * 2 * sizeof(u64), hipMemcpyDeviceToDevice, s));
                RCCL_OK(rccl().all_gather(m->pad.p, m->allp.p, (size_t)mx * 2, ncclUint64, m->comm, s));
                collective_done(m);
                allp = m->allp.as<u64>();
            }
            check_rc(cc_shard_finish(c, allp, (int64_t)(world * mx), labels_dev, res));
            res->n_labels = total + 1;
            res->max_id = total;
        } catch (const CCError& e) {
            abort_comm(m, e.msg);
            throw;
        } catch (const std::exception& e) {
            abort_comm(m, e.what());
            throw;
        }
    })
}

}  // extern "C"
