"""The sharded C entry with RCCL inside the library (cc_comm_* / cc_label_volume_sharded,
include/cc_mi355x.h): a ctypes caller shards without torch.distributed.  One rank per GPU; the
one-GPU box runs one rank (RCCL refuses two ranks on one device), through both schedules, against
the oracle on the whole volume."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _run(shape, bs, mode, mask=False, calls=2):
    import torch
    from cluster_tools_amd import _lib
    x = O.boundary_map(shape, origin=(4, 1, 2))
    m = None
    if mask:
        from oracle.synth import ellipsoid_mask
        m = ellipsoid_mask(shape)
    ref = O.label_volume(x, bs, 0.5, mode, m, n_threads=8)
    uid = _lib.comm_unique_id()
    assert len(uid) == 128
    with _lib.Comm(uid, 1, 0, 0) as comm, _lib.Context(0) as ctx:
        xd = torch.from_numpy(x).cuda()
        md = None if m is None else torch.from_numpy(m).cuda()
        for _ in range(calls):                 # the second call reuses the agreed schedule and buffers
            lab, res = ctx.label_volume_sharded(comm, xd, shape, 0, bs, 0.5, mode, mask=md)
            np.testing.assert_array_equal(lab.cpu().numpy().view(np.uint64), ref['labels'])
            assert res['n_labels'] == ref['n_labels'] and res['max_id'] == ref['n_labels'] - 1
            np.testing.assert_array_equal(ctx.lut(res['n_labels']), ref['lut'])


@pytest.mark.parametrize('mode', ['greater', 'less'])
def test_sharded_c_entry_one_rank(mode):
    """The one-read-back schedule with RCCL collectives on the context's stream."""
    _run((64, 150, 200), (16, 64, 64), mode)


def test_sharded_c_entry_mask():
    _run((48, 130, 170), (16, 64, 64), 'greater', mask=True)


def test_sharded_c_entry_synchronised(monkeypatch):
    """CC_FAST=0 (cc_shard_dev_ok = 0 on the context): the ranks agree on the host-synchronised
    schedule with uint64 seam planes; odd block shapes (no cube form) take it too."""
    monkeypatch.setenv('CC_FAST', '0')
    _run((64, 150, 200), (16, 64, 64), 'less')
    monkeypatch.delenv('CC_FAST')
    _run((45, 130, 170), (15, 45, 63), 'greater', calls=1)


def test_sharded_c_entry_errors():
    import torch
    from cluster_tools_amd import _lib
    uid = _lib.comm_unique_id()
    with _lib.Comm(uid, 1, 0, 0) as comm, _lib.Context(0) as ctx:
        x = torch.zeros((20, 32, 32), dtype=torch.float32, device='cuda')
        with pytest.raises(RuntimeError, match='block faces'):
            ctx.label_volume_sharded(comm, x, (40, 32, 32), 5, (16, 32, 32), 0.5)
        # a contiguous view one float into its storage: refused, not read with 16-B loads
        xo = torch.zeros(20 * 32 * 32 + 1, dtype=torch.float32, device='cuda')[1:].view(20, 32, 32)
        with pytest.raises(RuntimeError, match='16-byte aligned'):
            ctx.label_volume_sharded(comm, xo, (20, 32, 32), 0, (16, 32, 32), 0.5)
        lab, res = ctx.label_volume_sharded(comm, x, (20, 32, 32), 0, (16, 32, 32), 0.5)   # still usable
        ref = O.label_volume(np.zeros((20, 32, 32), np.float32), (16, 32, 32), 0.5, 'greater', None, n_threads=1)
        np.testing.assert_array_equal(lab.cpu().numpy().view(np.uint64), ref['labels'])
        assert res['n_labels'] == ref['n_labels']


def test_integration_comm_binding_runs_as_documented():
    """INTEGRATION.md's torch-free sharded binding (cc_comm_* + cc_label_volume_sharded) executed
    as written, one rank, against the oracle on the whole volume."""
    import ctypes
    import torch
    from conftest import exec_integration_binding, integration_blocks
    ns = exec_integration_binding()
    for b in integration_blocks():
        if 'def label_slab' in b:
            exec(compile(b, 'INTEGRATION.md', 'exec'), ns)
    shape, bs = (64, 150, 200), (16, 64, 64)
    x = O.boundary_map(shape, origin=(4, 1, 2))
    ref = O.label_volume(x, bs, 0.5, 'greater', None, n_threads=8)
    L = ns['_L']
    ctx = ctypes.c_void_p()
    assert L.cc_create(0, ctypes.byref(ctx)) == 0
    try:
        xd = torch.from_numpy(x).cuda()
        out = torch.empty(shape, dtype=torch.int64, device='cuda')
        torch.cuda.synchronize()
        res = ns['label_slab'](ctx, ns['rccl_id'](), 1, 0, 0, xd.data_ptr(), shape, 0, shape[0], bs, 0.5, 0,
                               out.data_ptr())
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint64), ref['labels'])
        assert res.n_labels == ref['n_labels'] and res.max_id == ref['n_labels'] - 1
    finally:
        L.cc_destroy(ctx)
