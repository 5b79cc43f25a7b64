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
// The same decisions as distributed.ShardedLabeler, on every rank alike: the schedule is agreed
// as the minimum of cc_shard_dev_ok over the ranks; a step whose status carries redo flags is
// relabelled synchronised; RF_PAIRS raises the pair capacity, RF_BIG / RF_CUBES / RF_IOVF leave
// the one-read-back schedule for good (properties of the input).
//
// RCCL is opened at the first cc_comm call (dlopen): the library itself needs no RCCL to load,
// and inside a process that already holds one (torch's), that copy is reused.
#include <dlfcn.h>

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
};

const RcclApi& rccl() {
    static RcclApi api;
    static std::once_flag once;
    static std::string err;
    std::call_once(once, [] {
        void* h = nullptr;
        if (const char* p = std::getenv("CC_RCCL_PATH"); p && *p) h = dlopen(p, RTLD_NOW | RTLD_LOCAL);
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

}  // namespace

struct cc_comm {
    ncclComm_t comm = nullptr;
    int world = 1, rank = 0, device = 0;
    hipStream_t stream = nullptr;          // used when the context has no stream of its own
    int64_t pair_cap = 2048;               // seam pairs per slab of the one-read-back buffers
    std::map<cc_ctx*, int> schedule;       // per context: 1 one-read-back, 0 synchronised (agreed)
    DevBuf sum, sums, top, upper, hdr, all, h8, bottom, top64, upper64, pairs, pad, allp;
};

static uint64_t next_pow2_u64(uint64_t n) {
    uint64_t p = 1;
    while (p < n) p <<= 1;
    return p;
}

// the context's stream for the call: the caller's (cc_set_stream), else the communicator's own
// (RCCL is given a real stream, never the null stream)
struct CommStream {
    cc_ctx* c;
    hipStream_t saved;
    CommStream(cc_ctx* c_, cc_comm* m) : c(c_), saved(c_->stream) {
        if (!c->stream) c->stream = m->stream;
    }
    ~CommStream() { c->stream = saved; }
};

// allgather of one uint64 per rank through device memory (host values, one synchronisation)
static std::vector<uint64_t> allgather_u64(cc_ctx* c, cc_comm* m, uint64_t v) {
    hipStream_t s = cstream(c);
    m->h8.ensure((1 + (size_t)m->world) * sizeof(u64));
    u64* d = m->h8.as<u64>();
    HIP_OK(hipMemcpyAsync(d, &v, sizeof(u64), hipMemcpyHostToDevice, s));
    RCCL_OK(rccl().all_gather(d, d + 1, 1, ncclUint64, m->comm, s));
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
}

static void check_rc(int rc) {
    if (rc < 0) throw CCError{g_err};
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
        ncclUniqueId uid;
        std::memcpy(&uid, id, sizeof(uid));
        try {
            HIP_OK(hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking));
            RCCL_OK(rccl().init_rank(&m->comm, world, uid, rank));
        } catch (...) {
            if (m->stream) (void)hipStreamDestroy(m->stream);
            delete m;
            throw;
        }
        *out = m;
    })
}

void cc_comm_destroy(cc_comm* m) {
    if (!m) return;
    (void)hipSetDevice(m->device);
    if (m->stream) (void)hipStreamSynchronize(m->stream);
    DevBuf* bufs[] = {&m->sum, &m->sums, &m->top, &m->upper, &m->hdr, &m->all, &m->h8, &m->bottom, &m->top64,
                      &m->upper64, &m->pairs, &m->pad, &m->allp};
    for (DevBuf* b : bufs) b->release();
    if (m->comm) (void)rccl().destroy(m->comm);
    if (m->stream) (void)hipStreamDestroy(m->stream);
    delete m;
}

int cc_label_volume_sharded(cc_ctx* c, cc_comm* m, const float* slab_dev, const uint8_t* mask_dev,
                            const int64_t global_shape[3], int64_t z_offset, int64_t slab_depth,
                            const int64_t block_shape[3], double threshold, int mode, uint64_t* labels_dev,
                            cc_result* res) {
    CC_TRY({
        CC_REQUIRE(c && m && slab_dev && global_shape && block_shape && labels_dev && res, "NULL argument");
        CC_REQUIRE(c->device == m->device, "context and communicator on different devices");
        CC_REQUIRE(slab_depth >= 1 && z_offset >= 0 && z_offset + slab_depth <= global_shape[0], "bad slab");
        CC_REQUIRE(z_offset % block_shape[0] == 0 && (slab_depth % block_shape[0] == 0 || z_offset + slab_depth == global_shape[0]),
                   "slabs must start and end on block faces");
        HIP_OK(hipSetDevice(c->device));
        CommStream cs(c, m);
        hipStream_t s = cstream(c);
        const int world = m->world, rank = m->rank;
        const int64_t Y = global_shape[1], X = global_shape[2];
        const int64_t slab[3] = {slab_depth, Y, X};
        const int64_t nby = (Y + block_shape[1] - 1) / block_shape[1], nbx = (X + block_shape[2] - 1) / block_shape[2];
        const bool cubes_ok = (nby == 1 || block_shape[1] % 2 == 0) && (nbx == 1 || block_shape[2] % 2 == 0);
        // the schedule, agreed over the ranks once per context (minimum of cc_shard_dev_ok)
        auto it = m->schedule.find(c);
        if (it == m->schedule.end()) {
            const auto oks = allgather_u64(c, m, cubes_ok && fast_ok(c) ? 1u : 0u);
            uint64_t all_ok = 1;
            for (uint64_t v : oks) all_ok &= v;
            it = m->schedule.emplace(c, (int)all_ok).first;
        }
        if (it->second) {
            const int64_t ncube = ((Y + 1) / 2) * ((X + 1) / 2);
            const int64_t cap = m->pair_cap;
            m->sum.ensure(sizeof(u64));
            m->sums.ensure(world * sizeof(u64));
            m->top.ensure(ncube * sizeof(u32));
            m->upper.ensure(ncube * sizeof(u32));
            m->hdr.ensure((cap + 1) * 2 * sizeof(u64));
            m->all.ensure((size_t)world * (cap + 1) * 2 * sizeof(u64));
            u64* sums = m->sums.as<u64>();
            check_rc(cc_shard_dev_begin(c, slab_dev, mask_dev, slab, block_shape, threshold, mode, z_offset, m->sum.as<u64>()));
            RCCL_OK(rccl().all_gather(m->sum.p, sums, 1, ncclUint64, m->comm, s));
            check_rc(cc_shard_dev_assign(c, sums, rank, world));
            if (rank + 1 < world) check_rc(cc_shard_dev_top_cubes(c, m->top.as<u32>()));
            shift_up(m, s, m->top.p, m->upper.p, (size_t)ncube, ncclUint32);
            check_rc(cc_shard_dev_seam_pairs(c, rank > 0 ? m->upper.as<u32>() : nullptr, sums, rank, m->hdr.as<u64>(), cap));
            RCCL_OK(rccl().all_gather(m->hdr.p, m->all.p, (size_t)(cap + 1) * 2, ncclUint64, m->comm, s));
            uint64_t status[4] = {0, 0, 0, 0};
            check_rc(cc_shard_dev_finish(c, m->all.as<u64>(), world, cap, sums, labels_dev, res, status));
            if (!status[0]) return 0;
            // every rank reads the same flags (computed from the allgathered headers and sums)
            if (status[0] & RF_PAIRS) m->pair_cap = (int64_t)next_pow2_u64(2 * status[1]);
            if (status[0] & (RF_BIG | RF_CUBES | RF_IOVF)) it->second = 0;
        }
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
            allp = m->allp.as<u64>();
        }
        check_rc(cc_shard_finish(c, allp, (int64_t)(world * mx), labels_dev, res));
        res->n_labels = total + 1;
        res->max_id = total;
    })
}

}  // extern "C"
