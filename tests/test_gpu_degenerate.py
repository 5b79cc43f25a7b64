"""Degenerate geometries against the oracle: volumes one voxel thick along an axis, blocks one
voxel thick, a single voxel, blocks larger than the volume, tiles truncated to one row / plane /
column everywhere (tile_info, the cube form of faces, the seams of one-voxel-thick tiles), both
modes, with and without a mask, and both single-volume schedules."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

CASES = [
    ((1, 40, 50), (1, 16, 16)),
    ((1, 1, 1), (1, 1, 1)),
    ((1, 1, 200), (1, 1, 64)),
    ((5, 1, 70), (2, 1, 33)),
    ((7, 9, 1), (3, 4, 1)),
    ((2, 3, 130), (1, 2, 64)),
    ((3, 70, 2), (3, 70, 2)),
    ((9, 11, 13), (64, 64, 64)),        # one block larger than the volume
    ((17, 33, 65), (1, 33, 65)),        # one-plane blocks
]


def _inputs(shape, seed):
    rng = np.random.default_rng(seed)
    x = rng.random(shape, dtype=np.float32)
    x[rng.random(shape) < 0.05] = 0.5    # ties with the threshold's normalised value
    m = (rng.random(shape) < 0.7).astype(np.uint8)
    return x, m


@pytest.mark.parametrize('fast', ['0', '1'])
@pytest.mark.parametrize('masked', [False, True])
@pytest.mark.parametrize('shape,bs', CASES)
def test_degenerate_vs_oracle(ctx, monkeypatch, shape, bs, masked, fast):
    import torch
    monkeypatch.setenv('CC_FAST', fast)
    x, m = _inputs(shape, sum(shape) + 7 * sum(bs))
    if not masked:
        m = None
    for mode in ('greater', 'less'):
        ref = O.label_volume(x, bs, 0.5, mode, m, n_threads=1)
        lab, res = ctx.label_volume(torch.from_numpy(x).cuda(), bs, 0.5, mode,
                                    mask=None if m is None else torch.from_numpy(m).cuda())
        np.testing.assert_array_equal(lab.cpu().numpy().view(np.uint64), ref['labels'])
        assert res['n_labels'] == ref['n_labels']
        np.testing.assert_array_equal(ctx.block_values(len(ref['values'])), ref['values'])


SHARDED = [
    ((17, 33, 65), (1, 33, 65), 3),     # one-plane blocks and slabs
    ((5, 1, 70), (2, 1, 33), 2),        # odd block x: no cube form, the synchronised schedule
    ((2, 3, 130), (1, 2, 64), 2),
    ((7, 9, 1), (3, 4, 1), 3),          # the last slab one plane thick
]


@pytest.mark.parametrize('schedule', [None, 'sync'])
@pytest.mark.parametrize('shape,bs,n', SHARDED)
def test_degenerate_sharded_vs_oracle(shape, bs, n, schedule):
    """The z-slab schedule over the same kinds of geometry (slabs of one plane, rows of one
    voxel), in one process, against the oracle on the whole volume."""
    import torch
    from cluster_tools_amd import _lib
    from cluster_tools_amd.distributed import label_slabs_single_process, assemble_lut
    x, m = _inputs(shape, 3 * sum(shape))
    for mask in (None, m):
        ref = O.label_volume(x, bs, 0.5, 'less', mask, n_threads=1)
        ctxs = [_lib.Context(0) for _ in range(n)]
        try:
            lab, res, sums, luts = label_slabs_single_process(
                ctxs, torch.from_numpy(x).cuda(), bs, 0.5, 'less',
                mask=None if mask is None else torch.from_numpy(mask).cuda(), schedule=schedule)
            np.testing.assert_array_equal(lab.cpu().numpy().view(np.uint64), ref['labels'])
            np.testing.assert_array_equal(assemble_lut(luts, sums), ref['lut'])
        finally:
            for c in ctxs:
                c.close()
