"""The library's sharded C entry (cc_label_volume_sharded) at world 2 and 3 on the one GPU of a
test box: every rank is its own process on cuda:0, the collectives are served by the test-only
RCCL stand-in tests/fake_rccl (CC_RCCL_PATH, shared-memory staging; RCCL itself refuses two ranks
on one device).  This runs the multi-rank branches the one-rank RCCL tests cannot reach -- the
seam planes shifted to rank + 1, rank > 0 seam pairs, the pair allgather, the status-driven redo,
the per-call agreement and the abort path -- against the oracle on the whole volume.
(Reference analogue: the job pool of /root/reference/cluster_tools/cluster_tasks.py:529-551.)"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FAKE = os.path.join(ROOT, 'tests', 'fake_rccl', 'libfake_rccl.so')
SHAPE, ORIGIN = (64, 150, 200), (4, 1, 2)


def _unique_id():
    import ctypes
    assert os.path.exists(FAKE), 'tests/fake_rccl/libfake_rccl.so not built (__graft_entry__.build())'
    buf = ctypes.create_string_buffer(128)
    assert ctypes.CDLL(FAKE).ncclGetUniqueId(buf) == 0
    return buf.raw.hex()


def _run(tmp_path, world, calls, mode='greater', mask=False, env_by_rank=None, env=None, calls_by_rank=None,
         shape=SHAPE, origin=ORIGIN, extra=None, timeout=240):
    """Start `world` worker processes (one rank each, all on cuda:0) and return their call logs."""
    uid = _unique_id()
    procs, outs = [], []
    for r in range(world):
        e = dict(os.environ, CC_RCCL_PATH=FAKE, CC_FAKE_RCCL_DIR=str(tmp_path), CC_FAKE_RCCL_TIMEOUT='60',
                 CC_COMM_TIMEOUT='60')
        e.update(env or {})
        e.update((env_by_rank or {}).get(r, {}))
        spec = dict(out=str(tmp_path), rank=r, world=world, uid=uid, shape=list(shape), origin=list(origin),
                    mode=mode, mask=mask, calls=(calls_by_rank or {}).get(r, calls), **(extra or {}))
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, 'tests', '_comm_worker.py'), json.dumps(spec)],
                                      env=e, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    try:
        for p in procs:
            outs.append(p.communicate(timeout=timeout)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for r, p in enumerate(procs):
        assert p.returncode == 0, 'rank %d: %s' % (r, outs[r][-4000:])
    return [json.load(open(str(tmp_path / ('rank%d.json' % r))))['calls'] for r in range(world)]


def _reference(block_shape, mode, mask=False):
    m = None
    if mask:
        from oracle.synth import ellipsoid_mask
        m = ellipsoid_mask(SHAPE)
    return O.label_volume(O.boundary_map(SHAPE, origin=ORIGIN), block_shape, 0.5, mode, m, n_threads=8)


def _check_call(tmp_path, logs, k, block_shape, mode, schedule, mask=False):
    ref = _reference(block_shape, mode, mask)
    world = len(logs)
    for r in range(world):
        e = logs[r][k]
        assert e['ok'], 'rank %d call %d: %s' % (r, k, e.get('error'))
        assert e['res']['n_labels'] == ref['n_labels'] and e['res']['max_id'] == ref['n_labels'] - 1
        assert e['info']['schedule'] == schedule, (r, k, e['info'])
    got = np.concatenate([np.load(str(tmp_path / ('rank%d_call%d.npy' % (r, k)))) for r in range(world)])
    np.testing.assert_array_equal(got.view(np.uint64), ref['labels'])


@pytest.mark.parametrize('world,mode,mask', [(2, 'greater', False), (3, 'less', True), (3, 'greater', False)])
def test_ranks_one_read_back(tmp_path, world, mode, mask):
    """The one-read-back schedule at world 2 / 3: sums allgather, cube-form seam planes to
    rank + 1, pair-buffer allgather; twice on the same communicator (buffers reused)."""
    bs = [16, 64, 64]
    logs = _run(tmp_path, world, [dict(block_shape=bs), dict(block_shape=bs)], mode=mode, mask=mask)
    for k in range(2):
        _check_call(tmp_path, logs, k, bs, mode, 'one-read-back', mask)


def test_ranks_pair_capacity_redo(tmp_path):
    """Seam-pair buffers of ONE pair (CC_SHARD_PAIR_CAP=1): the first step's status carries RF_PAIRS
    on every rank, the step is relabelled synchronised; the capacity grows and the second step
    runs the one-read-back schedule."""
    bs = [16, 64, 64]
    logs = _run(tmp_path, 3, [dict(block_shape=bs), dict(block_shape=bs)], mode='less', env={'CC_SHARD_PAIR_CAP': '1'})
    _check_call(tmp_path, logs, 0, bs, 'less', 'synchronised')
    _check_call(tmp_path, logs, 1, bs, 'less', 'one-read-back')
    for r in range(3):
        assert logs[r][0]['info']['redo'] & 8          # RF_PAIRS
        assert logs[r][1]['info']['pair_cap'] > 1 and logs[r][1]['info']['redo'] == 0


def test_ranks_one_rank_forces_synchronised(tmp_path):
    """CC_FAST=0 on rank 1 only: the agreement takes the minimum, every rank runs the
    host-synchronised schedule (uint64 seam planes, padded pair allgather)."""
    bs = [16, 64, 64]
    logs = _run(tmp_path, 2, [dict(block_shape=bs)], mode='greater', env_by_rank={1: {'CC_FAST': '0'}})
    _check_call(tmp_path, logs, 0, bs, 'greater', 'synchronised')


def test_ranks_block_shapes_change_on_one_communicator(tmp_path):
    """Even, odd, even block shapes through one context and communicator: the cube form is
    decided per call (odd block_shape[1:] -> synchronised), no stale schedule is reused."""
    calls = [dict(block_shape=[16, 64, 64]), dict(block_shape=[16, 45, 63]), dict(block_shape=[16, 64, 64])]
    logs = _run(tmp_path, 3, calls, mode='less')
    _check_call(tmp_path, logs, 0, [16, 64, 64], 'less', 'one-read-back')
    _check_call(tmp_path, logs, 1, [16, 45, 63], 'less', 'synchronised')
    _check_call(tmp_path, logs, 2, [16, 64, 64], 'less', 'one-read-back')


@pytest.mark.parametrize('shift,match', [(1, 'rank 1 rejected'), (16, 'do not tile')])
def test_ranks_bad_slab_on_one_rank(tmp_path, shift, match):
    """One rank's slab is wrong (off the block faces, or on a face but overlapping its neighbour):
    EVERY rank returns an error at the agreement, quickly, and the communicator stays usable --
    the next call is labelled correctly."""
    bs = [16, 64, 64]
    calls = [dict(block_shape=bs), dict(block_shape=bs)]
    logs = _run(tmp_path, 3, calls, calls_by_rank={1: [dict(block_shape=bs, z_shift=shift), dict(block_shape=bs)]})
    for r in range(3):
        e = logs[r][0]
        assert not e['ok'] and e['seconds'] < 20, (r, e)
        if r != 1 or shift != 1:
            assert match in e['error'], (r, e['error'])
        assert not e['info']['aborted']
    _check_call(tmp_path, logs, 1, bs, 'greater', 'one-read-back')


@pytest.mark.parametrize('fail_at', [2, 3])
def test_ranks_abort_after_a_collective(tmp_path, fail_at):
    """Rank 0 fails after its 2nd (sums allgather) or 3rd (seam-plane shift) collective of the
    step, with peers already inside the schedule: it aborts the communicator, the peers' pending
    collectives end with an error within seconds (not the timeout), every rank reports the
    communicator aborted, and the next call fails fast on every rank."""
    bs = [16, 64, 64]
    calls = [dict(block_shape=bs), dict(block_shape=bs)]
    logs = _run(tmp_path, 3, calls, env_by_rank={0: {'CC_COMM_FAIL_AT': str(fail_at)}})
    assert 'injected failure' in logs[0][0]['error']
    for r in range(3):
        e0, e1 = logs[r]
        assert not e0['ok'] and e0['seconds'] < 20, (r, e0)
        assert e0['info']['aborted'], (r, e0)
        assert not e1['ok'] and 'aborted' in e1['error'] and e1['seconds'] < 1, (r, e1)


@pytest.mark.parametrize('src', ['kernel', 'kernel_side'])
def test_ranks_input_from_an_unsynchronised_kernel(tmp_path, src):
    """The slab is written by a torch kernel queued behind ~50 ms of GPU sleep, and the call
    follows with no synchronisation: on torch's default stream the library's stream is fenced
    against it, on a side stream the wrapper binds that stream; either way the labels are right."""
    bs = [16, 64, 64]
    logs = _run(tmp_path, 2, [dict(block_shape=bs, src=src)], mode='greater')
    _check_call(tmp_path, logs, 0, bs, 'greater', 'one-read-back')


@pytest.mark.slow
@pytest.mark.parametrize('masked', [False, True])
def test_ranks_world8_c3_full_size(tmp_path, masked):
    """The 8-GPU strong-scaling split of BASELINE C3 (and of C4 = C3 + the ellipsoid uint8 mask)
    through the library's sharded C entry: eight rank processes (all on cuda:0, collectives by the
    stand-in), each labelling its (128, 2048, 2048) z-slab generated on the device, block
    (64, 512, 512); every slab's labels bit-exact (xxh64 of the raw uint64 labels) against the C
    oracle on the whole 1024 x 2048 x 2048 volume, n_labels equal, the one-read-back schedule on
    every rank."""
    import os as _os
    import torch
    import xxhash
    from cluster_tools_amd import _lib
    from cluster_tools_amd.synthetic import ellipsoid_mask_device
    shape, bs = (1024, 2048, 2048), [64, 512, 512]
    with _lib.Context(0) as ctx:
        x = ctx.generate_boundary_map(shape)
        inp = x.cpu().numpy()
        del x
        hmask = ellipsoid_mask_device(shape, 0, shape[0], torch.device('cuda', 0)).cpu().numpy() if masked else None
    torch.cuda.empty_cache()
    threads = max(1, min(16, len(_os.sched_getaffinity(0))))
    ref = O.label_volume(inp, bs, 0.5, 'greater', hmask, n_threads=threads, want_lut=False)
    del inp, hmask
    labels = ref.pop('labels')
    logs = _run(tmp_path, 8, [dict(block_shape=bs)], shape=shape, origin=(0, 0, 0), mask=masked,
                extra=dict(generate=True, hash_only=True), env={'CC_FAKE_RCCL_TIMEOUT': '300', 'CC_COMM_TIMEOUT': '300'},
                timeout=900)
    for r in range(8):
        e = logs[r][0]
        assert e['ok'], (r, e.get('error'))
        assert e['res']['n_labels'] == ref['n_labels'], (r, e['res'])
        assert e['info']['schedule'] == 'one-read-back', (r, e['info'])
        z0, zs = e['z0'], e['zs']
        assert (z0, zs) == (128 * r, 128)
        assert e['xxh64'] == xxhash.xxh64(labels[z0:z0 + zs].data).hexdigest(), 'rank %d labels differ' % r
    print("world 8 C3 label seconds per rank:", [round(logs[r][0]["label_seconds"], 3) for r in range(8)])


@pytest.mark.parametrize('shape,bs,world,mode,schedule', [
    ((33, 65, 129), (11, 13, 43), 3, 'greater', 'synchronised'),   # odd block y / x: no cube form
    ((20, 1, 300), (4, 1, 64), 2, 'less', 'one-read-back'),         # rows of one voxel in y
    ((45, 130, 170), (15, 45, 63), 3, 'less', 'synchronised'),
    ((9, 40, 2), (3, 40, 2), 3, 'greater', 'one-read-back'),        # slabs of 3 planes, 2-voxel rows
])
def test_ranks_geometries(tmp_path, shape, bs, world, mode, schedule):
    """Odd and degenerate geometries through the library's entry at world 2 / 3: each slab's labels
    against the oracle on the whole volume, the agreed schedule as the block shapes dictate."""
    origin = (2, 3, 5)
    logs = _run(tmp_path, world, [{'block_shape': list(bs)}], mode=mode, shape=shape, origin=origin)
    ref = O.label_volume(O.boundary_map(shape, origin=origin), bs, 0.5, mode, None, n_threads=8)
    for r in range(world):
        e = logs[r][0]
        assert e['ok'], 'rank %d: %s' % (r, e.get('error'))
        assert e['res']['n_labels'] == ref['n_labels']
        assert e['info']['schedule'] == schedule, (r, e['info'])
    got = np.concatenate([np.load(str(tmp_path / ('rank%d_call0.npy' % r))) for r in range(world)])
    np.testing.assert_array_equal(got.view(np.uint64), ref['labels'])
