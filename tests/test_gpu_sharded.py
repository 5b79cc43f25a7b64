"""The z-slab sharded path's device entry points (cc_shard_*), run for several slabs on one
GPU in one process (distributed.label_slabs_single_process), against the oracle on the
whole volume: raw uint64 labels and the assembled LUT must be identical."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('schedule', ['fast', 'sync'])
@pytest.mark.parametrize('n_slabs,shape,block_shape,mode', [
    (2, (64, 256, 256), (32, 128, 128), 'greater'),
    (2, (64, 256, 256), (32, 128, 128), 'less'),
    (4, (128, 200, 300), (32, 64, 128), 'less'),
    (3, (75, 130, 170), (25, 64, 64), 'greater'),
    (8, (64, 96, 160), (8, 48, 64), 'less'),
])
def test_sharded_single_gpu_vs_oracle(n_slabs, shape, block_shape, mode, schedule):
    """Both shard schedules: 'fast' = the one-read-back schedule (cc_shard_dev_*: sums, id
    bases and seam pairs stay on the device), 'sync' = the host-synchronised one."""
    import torch
    from cluster_tools_amd import _lib
    from cluster_tools_amd.distributed import label_slabs_single_process, assemble_lut
    x = O.boundary_map(shape, origin=(3, 0, 9))
    ctxs = [_lib.Context(0) for _ in range(n_slabs)]
    try:
        lab, res, sums, luts = label_slabs_single_process(ctxs, torch.from_numpy(x).cuda(), block_shape, 0.5, mode,
                                                          schedule=schedule)
        assert {r['schedule'] for r in res} == {'one-read-back' if schedule == 'fast' else 'synchronised'}
        ref = O.label_volume(x, block_shape, 0.5, mode, n_threads=8)
        np.testing.assert_array_equal(lab.cpu().numpy().view(np.uint64), ref['labels'])
        assert sum(sums) + 1 == ref['n_labels']
        np.testing.assert_array_equal(assemble_lut(luts, sums), ref['lut'])
        assert sum(r['n_components'] for r in res) == len(np.unique(ref['labels'])) - 1
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.parametrize('mode,block_shape', [('greater', (16, 64, 64)), ('less', (16, 64, 64)),
                                              ('less', (16, 45, 63))])   # odd: per-voxel u32 plane
def test_two_ranks_one_gpu_gloo(tmp_path, mode, block_shape):
    """The multi-process schedule (ShardedLabeler, one process per rank) with the real device
    work: two ranks share cuda:0, collectives over gloo staged through host memory (RCCL refuses
    two ranks on one device; the RCCL path differs only in TorchComm)."""
    import os
    import socket
    import subprocess
    import sys
    shape = (64, 150, 200)
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2',
           '--master-addr', '127.0.0.1', '--master-port', str(port),
           os.path.join(root, 'tests', '_sharded_worker.py'), str(tmp_path), mode,
           ','.join(map(str, shape)), ','.join(map(str, block_shape))]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    got = np.concatenate([np.load(str(tmp_path / ('slab_%d.npy' % k))) for k in range(2)]).astype(np.uint64)
    ref = O.label_volume(O.boundary_map(shape, n_threads=1), block_shape, 0.5, mode)
    np.testing.assert_array_equal(got, ref['labels'])
    for k in range(2):
        assert int(np.load(str(tmp_path / ('nl_%d.npy' % k)))[0]) == ref['n_labels']


def test_one_rank_rccl(tmp_path):
    """The production communicator (TorchComm over backend 'nccl' = RCCL, GPU tensors, device_id
    bound at init) through the whole ShardedLabeler schedule with one rank: the collectives
    (all_gather of counts and pairs) run on RCCL; the result equals the oracle's labelling."""
    import os
    import socket
    import subprocess
    import sys
    shape, block_shape = (48, 150, 200), (16, 64, 64)
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '1',
           '--master-addr', '127.0.0.1', '--master-port', str(port),
           os.path.join(root, 'tests', '_sharded_worker.py'), str(tmp_path), 'greater',
           ','.join(map(str, shape)), ','.join(map(str, block_shape)), 'nccl']
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    got = np.load(str(tmp_path / 'slab_0.npy')).astype(np.uint64)
    ref = O.label_volume(O.boundary_map(shape, n_threads=1), block_shape, 0.5, 'greater')
    np.testing.assert_array_equal(got, ref['labels'])
    assert int(np.load(str(tmp_path / 'nl_0.npy'))[0]) == ref['n_labels']


@pytest.mark.parametrize('n_slabs,mode,masked,form', [
    (4, 'less', True, None), (4, 'greater', False, None), (4, 'greater', True, 'voxel32'),
    # the 8-GPU strong-scaling split: 8 slabs of (128, 2048, 2048), seams every 128 planes
    (8, 'greater', True, None), (8, 'less', False, None)])
def test_sharded_c4_scale_vs_oracle(n_slabs, mode, masked, form):
    """SURVEY.md §8d parity at scale for the sharded configs: C4 (C3 + ellipsoid mask) over 4
    or 8 z-slabs on one GPU (8: the strong-scaling split of the 8-GPU run), with the cubes32 seam
    planes the ranks exchange over xGMI (or the per-voxel uint32 fallback), against the C oracle
    on the whole volume (6-connected seams: block_faces.py:87-113): raw labels identical
    (compared on the device), the assembled LUT identical, and the device contingency table of
    the two labellings a bijection (|unique(a, b)| == |unique(a)| == |unique(b)|)."""
    import os
    import torch
    from cluster_tools_amd import _lib
    from cluster_tools_amd.distributed import label_slabs_single_process, assemble_lut
    from cluster_tools_amd.synthetic import ellipsoid_mask_device
    shape, bs = (1024, 2048, 2048), (64, 512, 512)
    ctxs = [_lib.Context(0) for _ in range(n_slabs)]
    try:
        x = ctxs[0].generate_boundary_map(shape)
        mask = ellipsoid_mask_device(shape, 0, shape[0], x.device) if masked else None
        torch.cuda.synchronize()          # the mask is built on torch's stream, the ctx has its own
        b, res, sums, luts = label_slabs_single_process(ctxs, x, bs, 0.5, mode, mask=mask, form=form)
        inp = x.cpu().numpy()
        hmask = None if mask is None else mask.cpu().numpy()
        del x, mask
        threads = max(1, min(16, len(os.sched_getaffinity(0))))
        r = O.label_volume(inp, bs, 0.5, mode, hmask, n_threads=threads)
        del inp, hmask
        assert sum(sums) + 1 == r['n_labels']
        np.testing.assert_array_equal(assemble_lut(luts, sums), r['lut'])
        ref = torch.from_numpy(r.pop('labels').view(np.int64)).cuda()
        assert bool(torch.equal(b, ref))
        ev = ctxs[0].evaluate(ref, b, bs, ignore_label=None)
        n_comp = sum(q['n_components'] for q in res)
        assert ev['n_pairs'] == ev['n_seg_ids'] == ev['n_gt_ids'] == n_comp + 1
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.parametrize('order', ['0', '1'])
@pytest.mark.parametrize('mode', ['greater', 'less'])
def test_sharded_pass2_tile_order(monkeypatch, mode, order):
    """Both k_pass2 tile orders on the seam-map (z-slab) path against the oracle."""
    import torch
    from cluster_tools_amd import _lib
    from cluster_tools_amd.distributed import label_slabs_single_process, assemble_lut
    monkeypatch.setenv('CC_PASS2_ORDER', order)
    shape, bs = (96, 320, 448), (32, 128, 128)
    x = O.boundary_map(shape, origin=(1, 4, 7))
    ctxs = [_lib.Context(0) for _ in range(3)]
    try:
        lab, res, sums, luts = label_slabs_single_process(ctxs, torch.from_numpy(x).cuda(), bs, 0.5, mode)
        ref = O.label_volume(x, bs, 0.5, mode, n_threads=8)
        np.testing.assert_array_equal(lab.cpu().numpy().view(np.uint64), ref['labels'])
        np.testing.assert_array_equal(assemble_lut(luts, sums), ref['lut'])
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.slow
@pytest.mark.parametrize('mode', ['greater', 'less'])
def test_sharded_c5_geometry_vs_oracle(mode):
    """C5's seam geometry on one GPU: (256, 4096, 4096) as 2 z-slabs of (128, 4096, 4096), block
    (64, 512, 512), the 4096 x 4096 seam crossing as cubes32 planes (what the ranks send over xGMI),
    the z-fastest k_pass2 order (X >= 4096) -- raw labels and the assembled LUT bit-exact against
    the C oracle on the whole volume (reference face semantics: block_faces.py:87-113)."""
    import os
    import torch
    from cluster_tools_amd import _lib
    from cluster_tools_amd.distributed import label_slabs_single_process, assemble_lut
    shape, bs = (256, 4096, 4096), (64, 512, 512)
    ctxs = [_lib.Context(0) for _ in range(2)]
    try:
        x = ctxs[0].generate_boundary_map(shape)
        torch.cuda.synchronize()
        b, res, sums, luts = label_slabs_single_process(ctxs, x, bs, 0.5, mode, form='cubes32')
        inp = x.cpu().numpy()
        del x
        threads = max(1, min(16, len(os.sched_getaffinity(0))))
        r = O.label_volume(inp, bs, 0.5, mode, n_threads=threads)
        del inp
        assert sum(sums) + 1 == r['n_labels']
        np.testing.assert_array_equal(assemble_lut(luts, sums), r['lut'])
        ref = torch.from_numpy(r.pop('labels').view(np.int64)).cuda()
        assert bool(torch.equal(b, ref))
        del ref, b
        torch.cuda.empty_cache()
    finally:
        for c in ctxs:
            c.close()


def test_bench_self_launch_two_ranks_gloo():
    """`python bench.py --gpus 2 --workload c4` exactly as the driver's scaling run calls it (no
    torch.distributed.run around it): bench.py starts its two ranks itself; here both share
    cuda:0 with gloo collectives staged through host memory (CC_DIST_BACKEND=gloo; RCCL refuses
    two ranks on one device).  One JSON line with n_gpus 2, strong scaling over C4's volume."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, CC_DIST_BACKEND='gloo')
    env.pop('WORLD_SIZE', None)
    cmd = [sys.executable, os.path.join(root, 'bench.py'), '--gpus', '2', '--workload', 'c4', '--steps', '2',
           '--warmup', '1', '--no-cpu-baseline']
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d['n_gpus'] == 2 and d['scaling'] == 'strong' and d['config']['workload_id'] == 'c4'
    assert d['config']['shape'] == [1024, 2048, 2048] and d['config']['slab'] == [512, 2048, 2048]
    assert d['value'] > 0


def test_sharded_pair_capacity_redo():
    """Seam pair buffers too small (1 pair per slab): the status of the one-read-back step flags
    RF_PAIRS on every slab and the synchronised schedule relabels the step -- same labels."""
    import torch
    from cluster_tools_amd import _lib
    from cluster_tools_amd.distributed import label_slabs_single_process, assemble_lut
    shape, bs = (96, 160, 192), (16, 64, 64)
    x = O.boundary_map(shape, origin=(1, 2, 3))
    ctxs = [_lib.Context(0) for _ in range(3)]
    try:
        lab, res, sums, luts = label_slabs_single_process(ctxs, torch.from_numpy(x).cuda(), bs, 0.5, 'less', pair_cap=1)
        assert {r['schedule'] for r in res} == {'synchronised'}
        ref = O.label_volume(x, bs, 0.5, 'less', n_threads=8)
        np.testing.assert_array_equal(lab.cpu().numpy().view(np.uint64), ref['labels'])
        np.testing.assert_array_equal(assemble_lut(luts, sums), ref['lut'])
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.parametrize('env', [{'CC_FAST': '0'}, {'CC_FRONT_CHUNKS': '2'}])
def test_sharded_contexts_without_fast_schedule(monkeypatch, env):
    """Contexts that cannot run the one-read-back schedule (CC_FAST=0 forces the synchronised
    schedule; CC_FRONT_CHUNKS > 1 chunks the front): the sharded run asks cc_shard_dev_ok and
    takes the synchronised schedule instead of failing in cc_shard_dev_begin; schedule='fast' is
    refused with a clear error."""
    import torch
    from cluster_tools_amd import _lib
    from cluster_tools_amd.distributed import label_slabs_single_process, assemble_lut
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    shape, bs = (64, 150, 200), (16, 64, 64)
    x = O.boundary_map(shape, origin=(2, 1, 4))
    ctxs = [_lib.Context(0) for _ in range(3)]          # CC_FRONT_CHUNKS is read by cc_create
    try:
        assert not any(c.shard_dev_ok() for c in ctxs)
        xd = torch.from_numpy(x).cuda()
        lab, res, sums, luts = label_slabs_single_process(ctxs, xd, bs, 0.5, 'greater')
        assert {r['schedule'] for r in res} == {'synchronised'}
        ref = O.label_volume(x, bs, 0.5, 'greater', n_threads=8)
        np.testing.assert_array_equal(lab.cpu().numpy().view(np.uint64), ref['labels'])
        np.testing.assert_array_equal(assemble_lut(luts, sums), ref['lut'])
        with pytest.raises(ValueError, match='one-read-back'):
            label_slabs_single_process(ctxs, xd, bs, 0.5, 'greater', schedule='fast')
    finally:
        for c in ctxs:
            c.close()


def test_sharded_root_capacity_redo(monkeypatch):
    """More block-local roots than the contexts' root arrays hold (CC_ROOT_CAP=8) in the sharded
    one-read-back step: k_pass2 runs before the status is read, with slab sums beyond the LUT's
    allocation -- its LUT reads stay inside the allocation (lut_n) -- then RF_ROOTS sends the step
    to the synchronised schedule (same labels), and the grown capacity lets the next step run the
    one-read-back schedule."""
    import torch
    from cluster_tools_amd import _lib
    from cluster_tools_amd.distributed import label_slabs_single_process, assemble_lut
    monkeypatch.setenv('CC_ROOT_CAP', '8')
    shape, bs = (96, 160, 192), (16, 64, 64)
    x = O.boundary_map(shape, origin=(5, 2, 1))
    ref = O.label_volume(x, bs, 0.5, 'less', n_threads=8)
    ctxs = [_lib.Context(0) for _ in range(3)]
    try:
        xd = torch.from_numpy(x).cuda()
        for want in ('synchronised', 'one-read-back'):
            lab, res, sums, luts = label_slabs_single_process(ctxs, xd, bs, 0.5, 'less')
            assert {r['schedule'] for r in res} == {want}
            np.testing.assert_array_equal(lab.cpu().numpy().view(np.uint64), ref['labels'])
            np.testing.assert_array_equal(assemble_lut(luts, sums), ref['lut'])
    finally:
        for c in ctxs:
            c.close()
