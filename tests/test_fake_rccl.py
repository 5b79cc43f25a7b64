"""CPU checks of the test-only RCCL stand-in (tests/fake_rccl) that the multi-rank GPU tests of the
library's sharded C entry rely on (tests/test_gpu_comm_ranks.py): its protocol on host buffers
(CC_FAKE_RCCL_HOST=1) over 3 processes -- allgather, the grouped shift to rank + 1, abort
propagation, the timeout -- and that the product never loads it by default."""
import ctypes
import multiprocessing as mp
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FAKE = os.path.join(ROOT, 'tests', 'fake_rccl', 'libfake_rccl.so')
U64 = 5                                     # ncclUint64


class UniqueId(ctypes.Structure):            # ncclUniqueId, passed by value
    _fields_ = [('internal', ctypes.c_char * 128)]


def _lib():
    if not os.path.exists(FAKE):
        pytest.fail('tests/fake_rccl/libfake_rccl.so not built (__graft_entry__.build())')
    L = ctypes.CDLL(FAKE)
    P, I, S = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
    L.ncclCommInitRank.argtypes = [ctypes.POINTER(P), I, UniqueId, I]
    L.ncclAllGather.argtypes = [P, P, S, I, P, P]
    L.ncclSend.argtypes = [P, S, I, I, P, P]
    L.ncclRecv.argtypes = [P, S, I, I, P, P]
    L.ncclCommAbort.argtypes = [P]
    L.ncclCommDestroy.argtypes = [P]
    L.ncclGetErrorString.restype = ctypes.c_char_p
    return L


def _worker(uid, world, rank, what, q):
    os.environ['CC_FAKE_RCCL_HOST'] = '1'
    os.environ['CC_FAKE_RCCL_TIMEOUT'] = '3'
    L = _lib()
    comm = ctypes.c_void_p()
    idb = UniqueId.from_buffer_copy(uid)
    rc = L.ncclCommInitRank(ctypes.byref(comm), world, idb, rank)
    if rc:
        q.put((rank, 'init', rc))
        return
    out = {}
    if what == 'collectives':
        for it in range(3):                              # repeated: slots and mailboxes reused
            send = np.arange(4, dtype=np.uint64) + 100 * rank + 1000 * it
            recv = np.zeros(4 * world, dtype=np.uint64)
            assert L.ncclAllGather(send.ctypes.data, recv.ctypes.data, 4, U64, comm, None) == 0
            out['ag%d' % it] = recv.tolist()
            top = np.full(5, 7 * rank + it, dtype=np.uint64)
            upper = np.zeros(5, dtype=np.uint64)
            L.ncclGroupStart()
            if rank + 1 < world:
                assert L.ncclSend(top.ctypes.data, 5, U64, rank + 1, comm, None) == 0
            if rank > 0:
                assert L.ncclRecv(upper.ctypes.data, 5, U64, rank - 1, comm, None) == 0
            out['shift%d' % it] = int(L.ncclGroupEnd())
            out['upper%d' % it] = upper.tolist()
        L.ncclCommDestroy(comm)
    elif what == 'abort':
        if rank == 0:
            L.ncclCommAbort(comm)                       # rank 0 gives up before the allgather
            out['rc'] = 0
        else:
            send = np.zeros(1, dtype=np.uint64)
            recv = np.zeros(world, dtype=np.uint64)
            out['rc'] = int(L.ncclAllGather(send.ctypes.data, recv.ctypes.data, 1, U64, comm, None))
            out['msg'] = L.ncclGetErrorString(out['rc']).decode()
            L.ncclCommDestroy(comm)
    elif what == 'timeout':
        if rank == 0:
            out['rc'] = 0                               # rank 0 never joins the allgather
        else:
            send = np.zeros(1, dtype=np.uint64)
            recv = np.zeros(world, dtype=np.uint64)
            out['rc'] = int(L.ncclAllGather(send.ctypes.data, recv.ctypes.data, 1, U64, comm, None))
        L.ncclCommDestroy(comm)
    q.put((rank, what, out))


def _spawn(tmp_path, what, world=3):
    L = _lib()
    os.environ['CC_FAKE_RCCL_DIR'] = str(tmp_path)
    buf = ctypes.create_string_buffer(128)
    assert L.ncclGetUniqueId(buf) == 0
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(buf.raw, world, r, what, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict()
    for _ in range(world):
        r, w, out = q.get(timeout=60)
        assert w == what, (r, w, out)
        res[r] = out
    for p in ps:
        p.join(30)
        assert p.exitcode == 0
    assert not os.listdir(str(tmp_path)), 'the shared file is unlinked once every rank has mapped it'
    return res


def test_fake_rccl_collectives(tmp_path):
    res = _spawn(tmp_path, 'collectives')
    for it in range(3):
        want = [v for r in range(3) for v in (np.arange(4) + 100 * r + 1000 * it).tolist()]
        for r in range(3):
            assert res[r]['ag%d' % it] == want
            assert res[r]['shift%d' % it] == 0
            assert res[r]['upper%d' % it] == ([0] * 5 if r == 0 else [7 * (r - 1) + it] * 5)


def test_fake_rccl_abort_reaches_peers(tmp_path):
    res = _spawn(tmp_path, 'abort')
    for r in (1, 2):
        assert res[r]['rc'] == 6 and 'aborted' in res[r]['msg']    # ncclRemoteError


def test_fake_rccl_timeout(tmp_path):
    res = _spawn(tmp_path, 'timeout')
    for r in (1, 2):
        assert res[r]['rc'] == 2                                   # ncclSystemError after 3 s


def test_product_never_names_the_stand_in():
    """Only CC_RCCL_PATH (set by the multi-rank tests) can point the library at the stand-in."""
    for d, _, files in os.walk(os.path.join(ROOT, 'cluster_tools_amd')):
        for f in files:
            if f.endswith(('.py', '.hip', '.hpp', '.cpp')):
                txt = open(os.path.join(d, f), errors='replace').read()
                assert 'libfake_rccl' not in txt, f
    for f in ('bench.py', '__graft_entry__.py'):
        assert 'CC_RCCL_PATH' not in open(os.path.join(ROOT, f)).read()
