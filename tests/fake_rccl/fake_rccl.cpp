// fake_rccl.cpp -- TEST-ONLY stand-in for the nine RCCL entry points libcc_mi355x.so resolves
// (cluster_tools_amd/csrc/cc_comm.hip, rccl()), plus ncclCommAbort / ncclCommGetAsyncError.
//
// Why: the pool's GPU boxes have one MI355X and RCCL refuses two ranks on one device, so the
// multi-rank branches of cc_label_volume_sharded (shift_up of the seam planes, rank > 0 seam
// pairs, the padded pair allgather, the status-driven redo, the error paths) could not run before
// the driver's 8-GPU node.  This library lets 2..8 processes share cuda:0 as ranks of one
// "communicator": every collective is staged through a file-backed shared mapping (device -> host
// copy on the caller's stream, a barrier, host -> device copies), so it is exact but slow.
//
// It is loaded ONLY when a test sets CC_RCCL_PATH to it; nothing under cluster_tools_amd/ names it.
//
// Protocol (one mapping per communicator, named by the unique id's path):
//   header | world all-gather slots | world x world point-to-point mailboxes (each slot_bytes)
//   all-gather: own slot <- send; barrier; recv <- every slot; barrier (slots reusable)
//   send/recv : mailbox[src][dst] with posted / consumed counters (one message in flight)
// Every wait polls the abort word (ncclCommAbort of any rank) and a timeout
// (CC_FAKE_RCCL_TIMEOUT seconds, default 60): a peer that died or aborted makes the call return
// ncclRemoteError / ncclSystemError instead of hanging.
// CC_FAKE_RCCL_HOST=1 treats buffers as host memory (memcpy, no HIP): the CPU tests exercise the
// protocol itself without a GPU.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

namespace {

constexpr int kMaxRanks = 8;
constexpr size_t kHeader = 16384;

struct Header {
    std::atomic<uint32_t> attached;
    std::atomic<uint32_t> aborted;          // 1 + the aborting rank, 0 if none
    std::atomic<uint64_t> arrivals;         // monotonic barrier counter
    std::atomic<uint64_t> posted[kMaxRanks][kMaxRanks];
    std::atomic<uint64_t> consumed[kMaxRanks][kMaxRanks];
    uint64_t msg_bytes[kMaxRanks][kMaxRanks];
};
static_assert(sizeof(Header) <= kHeader, "header");

struct P2P {
    bool send;
    const void* sbuf;
    void* rbuf;
    size_t bytes;
    int peer;
    hipStream_t stream;
};

struct Comm {
    int world = 0, rank = 0;
    size_t slot = 0, map_bytes = 0;
    uint8_t* base = nullptr;
    uint64_t epoch = 0;                     // barriers this rank has passed
    ncclResult_t async_err = ncclSuccess;
    Header* hdr() const { return (Header*)base; }
    uint8_t* ag_slot(int r) const { return base + kHeader + (size_t)r * slot; }
    uint8_t* mailbox(int s, int d) const { return base + kHeader + (size_t)world * slot + ((size_t)s * world + d) * slot; }
};

thread_local int g_group = 0;
thread_local std::vector<P2P> g_ops;
thread_local Comm* g_group_comm = nullptr;

bool host_mode() {
    const char* e = std::getenv("CC_FAKE_RCCL_HOST");
    return e && *e == '1';
}

double timeout_s() {
    const char* e = std::getenv("CC_FAKE_RCCL_TIMEOUT");
    return e && *e ? std::atof(e) : 60.0;
}

double now_s() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

size_t type_size(ncclDataType_t t) {
    switch (t) {
        case ncclInt8: case ncclUint8: case ncclFloat8e4m3: case ncclFloat8e5m2: return 1;
        case ncclFloat16: case ncclBfloat16: return 2;
        case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
        case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
        default: return 0;
    }
}

// device <-> host copies, ordered on the caller's stream and complete on return
ncclResult_t to_host(void* dst, const void* src, size_t n, hipStream_t s) {
    if (host_mode()) { std::memcpy(dst, src, n); return ncclSuccess; }
    if (hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, s) != hipSuccess) return ncclUnhandledCudaError;
    return hipStreamSynchronize(s) == hipSuccess ? ncclSuccess : ncclUnhandledCudaError;
}

ncclResult_t to_dev(void* dst, const void* src, size_t n, hipStream_t s) {
    if (host_mode()) { std::memcpy(dst, src, n); return ncclSuccess; }
    if (hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, s) != hipSuccess) return ncclUnhandledCudaError;
    return hipStreamSynchronize(s) == hipSuccess ? ncclSuccess : ncclUnhandledCudaError;
}

// wait until pred() holds; a peer's abort or the timeout ends the wait with an error
template <class F>
ncclResult_t wait_for(Comm* c, F pred) {
    const double t0 = now_s(), limit = timeout_s();
    int spins = 0;
    while (!pred()) {
        if (c->hdr()->aborted.load()) { c->async_err = ncclRemoteError; return ncclRemoteError; }
        if (now_s() - t0 > limit) { c->async_err = ncclSystemError; return ncclSystemError; }
        if (++spins > 64) {
            timespec ts{0, 20000};
            nanosleep(&ts, nullptr);
        }
    }
    return ncclSuccess;
}

ncclResult_t barrier(Comm* c) {
    c->hdr()->arrivals.fetch_add(1);
    const uint64_t want = (c->epoch + 1) * (uint64_t)c->world;
    ncclResult_t r = wait_for(c, [&] { return c->hdr()->arrivals.load() >= want; });
    if (r == ncclSuccess) ++c->epoch;
    return r;
}

ncclResult_t usable(Comm* c) {
    if (!c || !c->base) return ncclInvalidArgument;
    if (c->async_err != ncclSuccess) return c->async_err;
    if (c->hdr()->aborted.load()) return c->async_err = ncclRemoteError;
    return ncclSuccess;
}

ncclResult_t do_send(Comm* c, const P2P& op) {
    Header* h = c->hdr();
    const int me = c->rank, d = op.peer;
    ncclResult_t r = wait_for(c, [&] { return h->consumed[me][d].load() == h->posted[me][d].load(); });
    if (r != ncclSuccess) return r;
    if ((r = to_host(c->mailbox(me, d), op.sbuf, op.bytes, op.stream)) != ncclSuccess) return r;
    h->msg_bytes[me][d] = op.bytes;
    h->posted[me][d].fetch_add(1);
    return ncclSuccess;
}

ncclResult_t do_recv(Comm* c, const P2P& op) {
    Header* h = c->hdr();
    const int me = c->rank, s = op.peer;
    ncclResult_t r = wait_for(c, [&] { return h->posted[s][me].load() > h->consumed[s][me].load(); });
    if (r != ncclSuccess) return r;
    if (h->msg_bytes[s][me] != op.bytes) return c->async_err = ncclInvalidUsage;   // size mismatch
    if ((r = to_dev(op.rbuf, c->mailbox(s, me), op.bytes, op.stream)) != ncclSuccess) return r;
    h->consumed[s][me].fetch_add(1);
    return ncclSuccess;
}

ncclResult_t run_ops(Comm* c, std::vector<P2P>& ops) {
    ncclResult_t r = ncclSuccess;
    for (const P2P& op : ops)          // sends first: a one-message mailbox never blocks a ring
        if (r == ncclSuccess && op.send) r = do_send(c, op);
    for (const P2P& op : ops)
        if (r == ncclSuccess && !op.send) r = do_recv(c, op);
    ops.clear();
    return r;
}

ncclResult_t p2p(bool send, const void* sbuf, void* rbuf, size_t count, ncclDataType_t dt, int peer, ncclComm_t comm,
                 hipStream_t stream) {
    Comm* c = (Comm*)comm;
    ncclResult_t r = usable(c);
    if (r != ncclSuccess) return r;
    const size_t bytes = count * type_size(dt);
    if (!type_size(dt) || peer < 0 || peer >= c->world || peer == c->rank || bytes > c->slot) return ncclInvalidArgument;
    P2P op{send, sbuf, rbuf, bytes, peer, stream};
    if (g_group > 0) {
        if (g_group_comm && g_group_comm != c) return ncclInvalidUsage;
        g_group_comm = c;
        g_ops.push_back(op);
        return ncclSuccess;
    }
    std::vector<P2P> one{op};
    return run_ops(c, one);
}

}  // namespace

extern "C" {

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
    static std::atomic<int> n{0};
    const char* dir = std::getenv("CC_FAKE_RCCL_DIR");
    if (!dir || !*dir) dir = "/tmp";
    std::memset(id, 0, sizeof(*id));
    timespec t;
    clock_gettime(CLOCK_REALTIME, &t);
    const int w = std::snprintf(id->internal, sizeof(id->internal), "%s/ccfake-%d-%d-%ld", dir, (int)getpid(),
                                n.fetch_add(1), (long)t.tv_nsec);
    return w > 0 && w < (int)sizeof(id->internal) ? ncclSuccess : ncclInvalidArgument;
}

ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
    if (!comm || nranks < 1 || nranks > kMaxRanks || rank < 0 || rank >= nranks) return ncclInvalidArgument;
    char path[sizeof(id.internal) + 1];
    std::memcpy(path, id.internal, sizeof(id.internal));
    path[sizeof(id.internal)] = 0;
    if (path[0] != '/') return ncclInvalidArgument;
    const char* e = std::getenv("CC_FAKE_RCCL_SLOT_MB");
    const size_t slot = (size_t)(e && *e ? std::atoi(e) : 8) << 20;
    const size_t bytes = kHeader + (size_t)nranks * slot + (size_t)nranks * nranks * slot;
    const int fd = open(path, O_RDWR | O_CREAT, 0600);
    if (fd < 0) return ncclSystemError;
    if (ftruncate(fd, (off_t)bytes) != 0) { close(fd); return ncclSystemError; }
    void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) return ncclSystemError;
    Comm* c = new Comm();
    c->world = nranks;
    c->rank = rank;
    c->slot = slot;
    c->map_bytes = bytes;
    c->base = (uint8_t*)p;
    c->hdr()->attached.fetch_add(1);
    ncclResult_t r = wait_for(c, [&] { return c->hdr()->attached.load() >= (uint32_t)nranks; });
    if (r == ncclSuccess) r = barrier(c);
    unlink(path);                           // every rank has it mapped: nothing is left on disk
    if (r != ncclSuccess) {
        munmap(c->base, c->map_bytes);
        delete c;
        return r;
    }
    *comm = (ncclComm_t)c;
    return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
    Comm* c = (Comm*)comm;
    if (!c) return ncclInvalidArgument;
    munmap(c->base, c->map_bytes);
    delete c;
    return ncclSuccess;
}

ncclResult_t ncclCommAbort(ncclComm_t comm) {
    Comm* c = (Comm*)comm;
    if (!c) return ncclInvalidArgument;
    uint32_t zero = 0;
    c->hdr()->aborted.compare_exchange_strong(zero, (uint32_t)c->rank + 1);
    munmap(c->base, c->map_bytes);
    delete c;
    return ncclSuccess;
}

ncclResult_t ncclCommGetAsyncError(ncclComm_t comm, ncclResult_t* err) {
    Comm* c = (Comm*)comm;
    if (!c || !err) return ncclInvalidArgument;
    *err = c->async_err != ncclSuccess ? c->async_err : (c->hdr()->aborted.load() ? ncclRemoteError : ncclSuccess);
    return ncclSuccess;
}

ncclResult_t ncclAllGather(const void* sendbuff, void* recvbuff, size_t sendcount, ncclDataType_t dt, ncclComm_t comm,
                           hipStream_t stream) {
    Comm* c = (Comm*)comm;
    ncclResult_t r = usable(c);
    if (r != ncclSuccess) return r;
    if (g_group > 0) return ncclInvalidUsage;            // not used inside groups by the library
    const size_t bytes = sendcount * type_size(dt);
    if (!type_size(dt) || bytes > c->slot) return ncclInvalidArgument;
    if ((r = to_host(c->ag_slot(c->rank), sendbuff, bytes, stream)) != ncclSuccess) return r;
    if ((r = barrier(c)) != ncclSuccess) return r;
    for (int k = 0; k < c->world && r == ncclSuccess; ++k)
        r = to_dev((uint8_t*)recvbuff + (size_t)k * bytes, c->ag_slot(k), bytes, stream);
    if (r != ncclSuccess) return r;
    return barrier(c);
}

ncclResult_t ncclSend(const void* sendbuff, size_t count, ncclDataType_t dt, int peer, ncclComm_t comm, hipStream_t stream) {
    return p2p(true, sendbuff, nullptr, count, dt, peer, comm, stream);
}

ncclResult_t ncclRecv(void* recvbuff, size_t count, ncclDataType_t dt, int peer, ncclComm_t comm, hipStream_t stream) {
    return p2p(false, nullptr, recvbuff, count, dt, peer, comm, stream);
}

ncclResult_t ncclGroupStart() {
    ++g_group;
    return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
    if (g_group <= 0) return ncclInvalidUsage;
    if (--g_group > 0) return ncclSuccess;
    Comm* c = g_group_comm;
    g_group_comm = nullptr;
    if (!c) return ncclSuccess;
    ncclResult_t r = usable(c);
    if (r != ncclSuccess) { g_ops.clear(); return r; }
    return run_ops(c, g_ops);
}

const char* ncclGetErrorString(ncclResult_t r) {
    switch (r) {
        case ncclSuccess: return "no error (fake_rccl)";
        case ncclUnhandledCudaError: return "HIP copy failed (fake_rccl)";
        case ncclSystemError: return "timed out waiting for a peer (fake_rccl)";
        case ncclInvalidArgument: return "invalid argument (fake_rccl)";
        case ncclInvalidUsage: return "invalid usage (fake_rccl)";
        case ncclRemoteError: return "a peer aborted the communicator (fake_rccl)";
        default: return "error (fake_rccl)";
    }
}

}  // extern "C"
