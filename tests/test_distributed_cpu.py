"""The z-slab schedule of cluster_tools_amd/distributed.py (collectives, id bases, seam exchange,
pair padding) over torch.distributed 'gloo' with world_size 2 and 3, on CPU.

The per-slab device work is stood in for by an oracle-backed fake context with the same
shard_* interface (the GPU implementation of those entry points is tested in
tests/test_gpu_sharded.py); the final labels must equal the oracle on the whole volume."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle as O


class FakeShardCtx:
    def __init__(self, dev_ok=True):
        self.dev_ok = dev_ok

    def shard_dev_ok(self):
        return self.dev_ok

    def shard_begin(self, x, block_shape, threshold, mode, z0, mask=None):
        r = O.label_volume(x.numpy(), block_shape, threshold, mode,
                           None if mask is None else mask.numpy())
        self.lab = r['labels'].astype(np.int64)
        return r['n_labels'] - 1

    def shard_assign(self, base):
        self.base = base
        self.lab[self.lab != 0] += base

    def shard_top_plane32(self, top32):
        t = self.lab[-1]
        top32.copy_(torch.from_numpy(np.where(t != 0, t - self.base + 1, 0).astype(np.int32)))

    def shard_top_cubes32(self, cubes):
        t = self.lab[-1]
        Y, X = t.shape
        p = np.zeros((2 * ((Y + 1) // 2), 2 * ((X + 1) // 2)), dtype=np.int64)
        p[:Y, :X] = t
        q = p.reshape(p.shape[0] // 2, 2, p.shape[1] // 2, 2)
        ids = q.max(axis=(1, 3))          # the foreground voxels of a cube share one component
        bits = sum(((q[:, j, :, i] != 0).astype(np.int64) << (2 * j + i)) for j in range(2) for i in range(2))
        w = np.where(ids != 0, ((ids - self.base + 1) << 4) | bits, 0)
        cubes.copy_(torch.from_numpy(w.astype(np.int32)))

    def seam_pairs_cubes32(self, cubes, upper_base, lower, pairs):
        c = cubes.numpy().astype(np.int64)
        Y, X = lower.shape
        yy, xx = np.meshgrid(np.arange(Y), np.arange(X), indexing='ij')
        e = c[yy // 2, xx // 2]
        on = (e >> ((yy & 1) * 2 + (xx & 1))) & 1
        up = np.where(on != 0, (e >> 4) - 1 + upper_base, 0)
        return self.seam_pairs(torch.from_numpy(up), lower, pairs)

    def seam_pairs32(self, upper32, upper_base, lower, pairs):
        u = upper32.numpy().astype(np.int64)
        return self.seam_pairs(torch.from_numpy(np.where(u != 0, u - 1 + upper_base, 0)), lower, pairs)

    def shard_planes(self, bottom=None, top=None):
        if bottom is not None:
            bottom.copy_(torch.from_numpy(self.lab[0]))
        if top is not None:
            top.copy_(torch.from_numpy(self.lab[-1]))

    def seam_pairs(self, upper, lower, pairs):
        a, b = upper.numpy().ravel(), lower.numpy().ravel()
        keep = (a != 0) & (b != 0)
        p = np.unique(np.stack([a[keep], b[keep]], axis=1), axis=0) if keep.any() else np.zeros((0, 2), np.int64)
        pairs[:len(p)] = torch.from_numpy(p)
        return len(p)

    # the one-read-back schedule's entry points (device buffers = CPU tensors here)
    def shard_dev_begin(self, x, block_shape, threshold, mode, z0, sum_t, mask=None):
        sum_t[0] = self.shard_begin(x, block_shape, threshold, mode, z0, mask)

    def shard_dev_assign(self, sums, rank, world):
        self.shard_assign(int(sums[:rank].sum()))

    def shard_dev_top_cubes(self, cubes):
        self.shard_top_cubes32(cubes)

    def shard_dev_seam_pairs(self, upper, sums, rank, hdr):
        cap = hdr.shape[0] - 1
        hdr.zero_()
        if upper is None:
            return
        Y, X = self.lab.shape[1:]
        tmp = torch.zeros((Y * X, 2), dtype=torch.int64)
        n = self.seam_pairs_cubes32(upper, int(sums[:rank - 1].sum()), torch.from_numpy(self.lab[0]), tmp)
        hdr[0, 0] = n
        m = min(n, cap)
        hdr[1:1 + m] = tmp[:m]

    def shard_dev_finish(self, all_, world, sums, out):
        from cluster_tools_amd import _lib
        cap = all_.shape[0] // world - 1
        bufs = all_.reshape(world, cap + 1, 2)
        counts = [int(b[0, 0]) for b in bufs]
        redo = 0
        for b in bufs:
            redo |= int(b[0, 1])
        if max(counts) > cap:
            redo |= _lib.RF_PAIRS
        n_labels = int(sums.sum()) + 1
        if redo:
            return {}, (redo, max(counts), n_labels, self.base)
        p = torch.cat([b[1:1 + c] for b, c in zip(bufs, counts)])
        res = self.shard_finish(p, p.shape[0], out)
        res['n_labels'] = n_labels
        return res, (0, max(counts), n_labels, self.base)

    def shard_finish(self, allp, n, out):
        mapping = {}
        if n:
            p = allp[:n].numpy()
            ids = np.unique(p)
            par = {int(i): int(i) for i in ids}

            def find(v):
                while par[v] != v:
                    par[v] = par[par[v]]
                    v = par[v]
                return v
            for a, b in p:
                ra, rb = find(int(a)), find(int(b))
                if ra != rb:
                    par[max(ra, rb)] = min(ra, rb)
            mapping = {i: find(i) for i in par}
        flat = self.lab.ravel()
        res = np.array([mapping.get(int(v), int(v)) for v in flat], dtype=np.int64).reshape(self.lab.shape)
        out.copy_(torch.from_numpy(res))
        return {'n_components': 0}


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _worker(rank, world, port, shape, block_shape, thr, mode, result_dir, form=None, pair_cap=None,
            no_dev_ranks=()):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from cluster_tools_amd.distributed import ShardedLabeler, TorchComm, slab_bounds

    class CountingComm(TorchComm):
        """The production communicator itself (no override of what it sends), with a call log."""
        calls = []

        def allgather_into(self, out, inp):
            self.calls.append('allgather_into')
            return TorchComm.allgather_into(self, out, inp)

        def shift_up(self, send, recv):
            self.calls.append('shift_up')
            return TorchComm.shift_up(self, send, recv)

        def allgather_int(self, v):
            self.calls.append('allgather_int')
            return TorchComm.allgather_int(self, v)

    x = O.boundary_map(shape, n_threads=1)
    z0, zs = slab_bounds(shape[0], block_shape[0], world)[rank]
    comm = CountingComm(device=None)
    lab = ShardedLabeler(FakeShardCtx(dev_ok=rank not in no_dev_ranks), shape, block_shape, z0, zs, device=None,
                         comm=comm, force_form=form)
    CountingComm.calls.clear()
    if pair_cap is not None:
        lab.pair_cap = pair_cap
    out = torch.empty((zs,) + tuple(shape[1:]), dtype=torch.int64)
    res = lab.label(torch.from_numpy(x[z0:z0 + zs].copy()), thr, mode, out=out)
    sched = [res['schedule']]
    if pair_cap is not None:              # a too-small pair buffer: the step was redone synchronised,
        res = lab.label(torch.from_numpy(x[z0:z0 + zs].copy()), thr, mode, out=out)   # the next fits
        sched.append(res['schedule'])
    np.save(os.path.join(result_dir, 'slab_%d.npy' % rank), out.numpy())
    np.save(os.path.join(result_dir, 'nl_%d.npy' % rank), np.array([res['n_labels'], res['id_base']]))
    with open(os.path.join(result_dir, 'sched_%d.txt' % rank), 'w') as f:
        f.write(' '.join(sched) + ' %d' % lab.pair_cap)
    with open(os.path.join(result_dir, 'calls_%d.txt' % rank), 'w') as f:
        f.write(' '.join(CountingComm.calls))
    dist.destroy_process_group()


@pytest.mark.parametrize('world,shape,block_shape,mode', [
    (2, (32, 70, 90), (16, 32, 32), 'greater'),
    (2, (32, 70, 90), (8, 40, 48), 'less'),
    (3, (40, 64, 64), (8, 32, 32), 'less'),
    (2, (32, 70, 90), (16, 32, 32), 'voxel32'),     # seam-plane fallbacks for slabs with many ids
    (3, (40, 64, 64), (8, 32, 32), 'voxel64'),
])
def test_gloo_sharded_schedule_matches_oracle(tmp_path, world, shape, block_shape, mode):
    port = _free_port()
    form = None
    if mode.startswith('voxel'):
        form, mode = mode, 'less'
    mp.spawn(_worker, args=(world, port, shape, block_shape, 0.5, mode, str(tmp_path), form), nprocs=world,
             join=True)
    got = np.concatenate([np.load(str(tmp_path / ('slab_%d.npy' % r))) for r in range(world)]).astype(np.uint64)
    ref = O.label_volume(O.boundary_map(shape, n_threads=1), block_shape, 0.5, mode)
    np.testing.assert_array_equal(got, ref['labels'])
    for r in range(world):
        assert int(np.load(str(tmp_path / ('nl_%d.npy' % r)))[0]) == ref['n_labels']
        sched = open(str(tmp_path / ('sched_%d.txt' % r))).read().split()
        # even y/x blocks and no forced form: the one-read-back schedule, else the synchronised one
        fast = form is None and block_shape[1] % 2 == 0 and block_shape[2] % 2 == 0
        assert sched[0] == ('one-read-back' if fast else 'synchronised')
        calls = open(str(tmp_path / ('calls_%d.txt' % r))).read().split()
        if fast:
            # the production communicator's stream-ordered collectives ran at world > 1: the sums'
            # allgather, the seam plane's point-to-point shift, the pair buffers' allgather
            assert calls == ['allgather_into', 'shift_up', 'allgather_into']
        else:
            assert 'shift_up' in calls and 'allgather_into' not in calls


@pytest.mark.parametrize('world', [2, 3])
def test_gloo_schedule_agreed_over_ranks(tmp_path, world):
    """One rank's context cannot run the one-read-back schedule (cc_shard_dev_ok = 0: CC_FAST=0,
    CC_FRONT_CHUNKS > 1, debug flags or the quirk option): every rank takes the synchronised one,
    so the collectives match, and the labels equal the oracle."""
    shape, block_shape = (40, 64, 64), (8, 32, 32)
    port = _free_port()
    mp.spawn(_worker, args=(world, port, shape, block_shape, 0.5, 'greater', str(tmp_path), None, None, (world - 1,)),
             nprocs=world, join=True)
    got = np.concatenate([np.load(str(tmp_path / ('slab_%d.npy' % r))) for r in range(world)]).astype(np.uint64)
    ref = O.label_volume(O.boundary_map(shape, n_threads=1), block_shape, 0.5, 'greater')
    np.testing.assert_array_equal(got, ref['labels'])
    for r in range(world):
        assert open(str(tmp_path / ('sched_%d.txt' % r))).read().split()[0] == 'synchronised'


def test_check_rccl_ranks():
    """bench.py / sharded_job.py fail fast when RCCL cannot give every local rank a GPU."""
    from cluster_tools_amd.distributed import check_rccl_ranks
    n = torch.cuda.device_count()
    check_rccl_ranks('gloo', 5, n + 8)             # gloo may share GPUs
    with pytest.raises(RuntimeError, match='one GPU per rank'):
        check_rccl_ranks('nccl', 0, n + 1)
    with pytest.raises(RuntimeError, match='one GPU per rank'):
        check_rccl_ranks('nccl', n, n + 1)
    if n:
        check_rccl_ranks('nccl', n - 1, n)


@pytest.mark.parametrize('world', [2, 3])
def test_gloo_pair_capacity_redo(tmp_path, world):
    """A pair buffer too small for the seams: every rank sees the same header counts, relabels the
    step with the synchronised schedule (same labels) and raises the capacity alike, so the next
    step runs the one-read-back schedule again."""
    shape, block_shape = (40, 64, 64), (8, 32, 32)
    port = _free_port()
    mp.spawn(_worker, args=(world, port, shape, block_shape, 0.5, 'less', str(tmp_path), None, 1), nprocs=world,
             join=True)
    got = np.concatenate([np.load(str(tmp_path / ('slab_%d.npy' % r))) for r in range(world)]).astype(np.uint64)
    ref = O.label_volume(O.boundary_map(shape, n_threads=1), block_shape, 0.5, 'less')
    np.testing.assert_array_equal(got, ref['labels'])
    caps = set()
    for r in range(world):
        s = open(str(tmp_path / ('sched_%d.txt' % r))).read().split()
        assert s[:2] == ['synchronised', 'one-read-back']
        caps.add(int(s[2]))
    assert len(caps) == 1 and caps.pop() > 1


def test_seam_form_choice():
    from cluster_tools_amd.distributed import ShardedLabeler as S
    assert S.seam_form(True, 2 ** 28 - 3) == 'cubes32'
    assert S.seam_form(True, 2 ** 28 - 2) == 'voxel32'
    assert S.seam_form(False, 5) == 'voxel32'
    assert S.seam_form(True, 2 ** 32 - 2) == 'voxel64'


def test_slab_bounds():
    from cluster_tools_amd.distributed import slab_bounds, check_slabs
    b = slab_bounds(1024, 64, 8)
    assert b == [(128 * r, 128) for r in range(8)]
    b = slab_bounds(125, 50, 2)
    assert b == [(0, 100), (100, 25)]
    for z0, zs in b:
        check_slabs((125, 10, 10), (50, 10, 10), z0, zs)
    with pytest.raises(ValueError):
        check_slabs((128, 4, 4), (64, 4, 4), 32, 64)
