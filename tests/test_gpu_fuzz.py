"""Seeded random cases of the fused path against the oracle: random volume and block shapes (odd
and even, blocks larger or smaller than tiles), thresholds, modes (greater / less / equal), input
kinds (the boundary map, its continuous variant, white noise, a few quantised levels with ties,
constant blocks, NaN / inf / -0.0 sprinkled in), with and without a mask (random, empty blocks,
all-zero), on both single-volume schedules.  Every case is bit-exact on labels, block values,
n_labels and the LUT."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

N_CASES = 72             # cases 48.. are larger (up to 130 x 330 x 430: many tiles and blocks)


def _case(i):
    rng = np.random.default_rng(1000 + i)
    hi = [70, 140, 200] if i < 48 else [130, 330, 430]
    shape = tuple(int(v) for v in rng.integers([1, 1, 1] if i < 48 else [20, 40, 40], hi))
    bs = tuple(int(min(s, v)) if rng.random() < 0.3 else int(v)
               for s, v in zip(shape, rng.integers([1, 1, 1], [h + 10 for h in hi])))
    kind = ['map', 'cont', 'noise', 'levels', 'const_blocks'][i % 5]
    if kind in ('map', 'cont'):
        x = O.boundary_map(shape, origin=tuple(int(v) for v in rng.integers(0, 50, 3)), n_threads=4,
                           dither=kind == 'cont')
    elif kind == 'noise':
        x = rng.random(shape, dtype=np.float32)
    elif kind == 'levels':
        x = (rng.integers(0, 5, shape) / 4.0).astype(np.float32)
    else:
        x = np.zeros(shape, np.float32)
        x[:, :, : shape[2] // 2] = float(rng.random())
        x[rng.random(shape) < 0.02] = float(rng.random())
    if i % 7 == 3:
        flat = x.reshape(-1)
        idx = rng.integers(0, flat.size, max(1, flat.size // 500))
        flat[idx] = rng.choice(np.array([np.nan, np.inf, -np.inf, -0.0], np.float32), len(idx))
    mk = i % 4
    if mk == 0:
        m = None
    elif mk == 1:
        m = (rng.random(shape) < 0.6).astype(np.uint8)
    elif mk == 2:
        m = np.zeros(shape, np.uint8)
        sl = tuple(slice(0, max(1, s // 2)) for s in shape)
        m[sl] = 1
    else:
        m = np.zeros(shape, np.uint8)
    mode = ['greater', 'less', 'equal'][i % 3]
    thr = float(rng.choice([0.5, 0.25, 0.75, float(rng.random())]))
    return x, bs, thr, mode, m


@pytest.mark.parametrize('fast', ['1', '0'])
@pytest.mark.parametrize('i', range(N_CASES))
def test_fuzz_vs_oracle(ctx, monkeypatch, i, fast):
    import torch
    monkeypatch.setenv('CC_FAST', fast)
    x, bs, thr, mode, m = _case(i)
    ref = O.label_volume(x, bs, thr, mode, m, n_threads=4)
    lab, res = ctx.label_volume(torch.from_numpy(x).cuda(), bs, thr, mode,
                                mask=None if m is None else torch.from_numpy(m).cuda())
    np.testing.assert_array_equal(lab.cpu().numpy().view(np.uint64), ref['labels'])
    assert res['n_labels'] == ref['n_labels'] and res['max_id'] == ref['max_id']
    np.testing.assert_array_equal(ctx.block_values(len(ref['values'])), ref['values'])
    np.testing.assert_array_equal(ctx.lut(res['n_labels']), ref['lut'])


@pytest.mark.parametrize('i', range(0, N_CASES, 3))
def test_fuzz_threshold_task_vs_oracle(ctx, i):
    """The Threshold task's entry (cc_threshold) on the same cases (no mask: the task has none)."""
    import torch
    x, bs, thr, mode, _ = _case(i)
    ref = O.threshold_volume(x, bs, thr, mode)
    out = ctx.threshold(torch.from_numpy(x).cuda(), bs, thr, mode)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)


@pytest.mark.parametrize('schedule', [None, 'sync'])
@pytest.mark.parametrize('i', range(1, N_CASES, 4))
def test_fuzz_sharded_vs_oracle(i, schedule):
    """The z-slab schedule in one process over 2-4 slabs of the same cases (as many as the block
    rows allow), against the oracle on the whole volume."""
    import torch
    from cluster_tools_amd import _lib
    from cluster_tools_amd.distributed import label_slabs_single_process, assemble_lut
    x, bs, thr, mode, m = _case(i)
    nbz = -(-x.shape[0] // bs[0])
    n = min(nbz, 2 + i % 3)
    if n < 2:
        pytest.skip('one block row: nothing to shard')
    ref = O.label_volume(x, bs, thr, mode, m, n_threads=4)
    ctxs = [_lib.Context(0) for _ in range(n)]
    try:
        lab, res, sums, luts = label_slabs_single_process(
            ctxs, torch.from_numpy(x).cuda(), bs, thr, mode,
            mask=None if m is None else torch.from_numpy(m).cuda(), schedule=schedule)
        np.testing.assert_array_equal(lab.cpu().numpy().view(np.uint64), ref['labels'])
        np.testing.assert_array_equal(assemble_lut(luts, sums), ref['lut'])
    finally:
        for c in ctxs:
            c.close()
