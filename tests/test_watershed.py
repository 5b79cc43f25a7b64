"""Seeded watershed per block (reference watershed/watershed_from_seeds.py:143-273, the
WatershedFromSeeds task of ThresholdAndWatershedWorkflow).  The reference's watershed call
(vu.watershed) does not exist in its volume_utils, so parity is UNPINNED: the device result
(cc_watershed_from_seeds) is checked bit-exactly against oracle/watershed.py, which restates the
job around the call and defines the watershed (minimax path cost, smallest label among the
optimal predecessors, 6-connected inside each block)."""
import numpy as np
import pytest

from oracle import oracle as O
from oracle import watershed as W


def test_oracle_ridge_and_plateau():
    """A line of voxels: two seeds, a ridge between them -> the split is at the ridge, the ridge
    voxel itself goes to the smaller label when both sides reach it at the same cost."""
    x = np.array([[[0.0, 0.2, 0.9, 0.3, 0.0]]], dtype=np.float32)
    s = np.array([[[5, 0, 0, 0, 7]]], dtype=np.uint64)
    assert W.watershed_block(x, s).tolist() == [[[5, 5, 5, 7, 7]]]
    x = np.array([[[0.0, 0.5, 0.5, 0.5, 0.0]]], dtype=np.float32)      # plateau: smaller label floods it
    assert W.watershed_block(x, s).tolist() == [[[5, 5, 5, 5, 7]]]
    s2 = np.array([[[9, 0, 0, 0, 3]]], dtype=np.uint64)
    assert W.watershed_block(x, s2).tolist() == [[[9, 3, 3, 3, 3]]]


def test_oracle_blocks_are_independent_and_masked():
    rng = np.random.default_rng(0)
    x = rng.random((8, 12, 16)).astype(np.float32)
    s = np.zeros(x.shape, dtype=np.uint64)
    s[0, 0, 0] = 4                                          # block (0,0,0) only
    out = W.watershed_from_seeds(x, s, (8, 12, 8))
    assert (out[:, :, :8] == 4).all() and (out[:, :, 8:] == 0).all()
    m = np.ones(x.shape, dtype=np.uint8)
    m[:, 6:, :] = 0
    out = W.watershed_from_seeds(x, s, (8, 12, 8), m)
    assert (out[:, :6, :8] == 4).all() and (out[:, 6:] == 0).all()


def _seeds_from_ccl(ctx, x, bs):
    """the workflow's seeds: the thresholded components ('less': cell interiors) of the input"""
    import torch
    lab, _ = ctx.label_volume(torch.from_numpy(x).cuda(), bs, 0.5, 'less')
    return lab


CASES = [((40, 72, 88), (16, 32, 32)), ((40, 72, 88), (40, 72, 88)), ((33, 65, 70), (11, 30, 40))]


@pytest.mark.gpu
@pytest.mark.parametrize('shape,bs', CASES)
def test_gpu_watershed_ccl_seeds_vs_oracle(ctx, shape, bs):
    """Seeds from the device CCL of a boundary map (the ThresholdAndWatershed chain), the map as
    input; ragged blocks and tiles; in place (out = seeds) as the workflow writes."""
    import torch
    x = O.boundary_map(shape, origin=(3, 5, 7))
    seeds = _seeds_from_ccl(ctx, x, bs)
    want = W.watershed_from_seeds(x, seeds.cpu().numpy().view(np.uint64), bs)
    xd = torch.from_numpy(x).cuda()
    got, rounds = ctx.watershed_from_seeds(xd, seeds, bs)
    np.testing.assert_array_equal(got.cpu().numpy().view(np.uint64), want)
    assert rounds >= 2
    ctx.watershed_from_seeds(xd, seeds, bs, out=seeds)                 # in place
    np.testing.assert_array_equal(seeds.cpu().numpy().view(np.uint64), want)


@pytest.mark.gpu
@pytest.mark.parametrize('kind', ['quantized', 'sparse_seeds', 'masked', 'nan_inf_blocks', 'big_ids'])
def test_gpu_watershed_cases_vs_oracle(ctx, kind):
    """Plateaus (quantized input: label ties), few seeds (long paths across many tiles), a mask
    (input 1 / output 0 outside it, an all-masked block), NaN / inf blocks, ids near 2^32."""
    import torch
    rng = np.random.default_rng(17)
    shape, bs = (24, 80, 100), (24, 40, 50)
    x = (rng.integers(0, 5, shape) / np.float32(4)).astype(np.float32)
    seeds = np.zeros(shape, dtype=np.uint64)
    idx = rng.integers(0, np.prod(shape), 300 if kind != 'sparse_seeds' else 6)
    seeds.reshape(-1)[idx] = rng.integers(1, 50, idx.size).astype(np.uint64)
    mask = None
    if kind == 'masked':
        mask = (rng.random(shape) < 0.8).astype(np.uint8)
        mask[:, :40, :50] = 0                                           # one block without mask voxels
    if kind == 'nan_inf_blocks':
        x[3, 5, 7] = np.nan                                             # block (0, 0, 0)
        x[10, 50, 70] = np.inf                                          # block (0, 1, 1)
        x[20, 10, 60] = -np.inf                                         # block (0, 0, 1)
    if kind == 'big_ids':
        seeds[seeds != 0] += np.uint64(2 ** 32 - 60)
    want = W.watershed_from_seeds(x, seeds, bs, mask)
    got, _ = ctx.watershed_from_seeds(torch.from_numpy(x).cuda(), torch.from_numpy(seeds.view(np.int64)).cuda(), bs,
                                      None if mask is None else torch.from_numpy(mask).cuda())
    np.testing.assert_array_equal(got.cpu().numpy().view(np.uint64), want)


@pytest.mark.gpu
def test_gpu_watershed_rejects_wide_ids(ctx):
    import torch
    x = torch.zeros((4, 8, 8), dtype=torch.float32, device='cuda')
    s = torch.zeros((4, 8, 8), dtype=torch.int64, device='cuda')
    s[0, 0, 0] = 2 ** 32 - 1
    with pytest.raises(RuntimeError, match='2\\^32'):
        ctx.watershed_from_seeds(x, s, (4, 8, 8))
