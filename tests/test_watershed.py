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


# ---- 4-D (channel) input: _read_data (watershed_from_seeds.py:127-139) ----
def _ws_read_cases():
    import json
    import os
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')
    with open(os.path.join(here, 'index_ws_read.json')) as f:
        idx = json.load(f)
    return here, sorted(idx.items())


WS_READ_HERE, WS_READ_CASES = _ws_read_cases()


def _ws_read_golden(name):
    import os
    d = np.load(os.path.join(WS_READ_HERE, 'ws_read_%s.npz' % name))
    return d['input'], d['expected']


@pytest.mark.parametrize('name,meta', WS_READ_CASES, ids=[c[0] for c in WS_READ_CASES])
def test_oracle_read_data_golden(name, meta):
    """oracle.watershed.read_data restates the reference's _read_data: equal (NaN-aware, bit for
    bit) to the reference's own output on every golden case."""
    x4, want = _ws_read_golden(name)
    got = W.read_data(x4, meta['block_shape'], meta['channel_begin'], meta['channel_end'], meta['agg'])
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize('name,meta', WS_READ_CASES, ids=[c[0] for c in WS_READ_CASES])
def test_gpu_normalize_channels_golden(ctx, name, meta):
    """cc_normalize_channels against the reference's _read_data output, bit for bit (the host
    casts to float32 first, as normalize's astype does; the channel range is sliced on the host,
    as the job's read does)."""
    import torch
    x4, want = _ws_read_golden(name)
    sel = np.ascontiguousarray(x4[meta['channel_begin']:meta['channel_end']].astype(np.float32))
    got = ctx.normalize_channels(torch.from_numpy(sel).cuda(), meta['block_shape'], meta['agg']).cpu().numpy()
    # bit for bit, except that a NaN's sign / payload is not pinned (numpy's SIMD np.max returns the
    # x86 default NaN, the mean path the propagated one; the watershed orders every NaN alike)
    nan = np.isnan(want)
    np.testing.assert_array_equal(np.isnan(got), nan)
    np.testing.assert_array_equal(got.view(np.uint32)[~nan], want.view(np.uint32)[~nan])


@pytest.mark.gpu
@pytest.mark.parametrize('shape,bs', [((10, 20, 44), (4, 8, 20)),      # rows of float4 (k_norm_agg4)
                                      ((10, 20, 45), (4, 8, 20)),      # X % 4 != 0: the element kernel
                                      ((10, 20, 44), (4, 8, 22))],     # block x % 4 != 0: the element kernel
                         ids=['rows4', 'odd_x', 'odd_block_x'])
@pytest.mark.parametrize('agg', ['mean', 'max', 'min'])
def test_gpu_normalize_channels_paths_vs_oracle(ctx, shape, bs, agg):
    """Both device kernels of cc_normalize_channels against oracle.watershed.read_data (NaN-aware,
    bit for bit), random channels of different scales with a NaN, an inf and a constant block."""
    import torch
    rng = np.random.default_rng(11)
    x4 = np.stack([rng.random(shape, dtype=np.float32) * np.float32(s) for s in (1.0, 1e3, 3e-3)])
    x4[1, 1, 2, 3] = np.nan
    x4[2, 9, 19, 40] = np.inf
    x4[:, 4:8, 8:16, :bs[2]] = np.float32(0.5)
    want = W.read_data(x4, bs, 0, None, agg)
    got = ctx.normalize_channels(torch.from_numpy(x4).cuda(), bs, agg).cpu().numpy()
    nan = np.isnan(want)
    np.testing.assert_array_equal(np.isnan(got), nan)
    np.testing.assert_array_equal(got.view(np.uint32)[~nan], want.view(np.uint32)[~nan])


@pytest.mark.gpu
@pytest.mark.parametrize('agg', ['mean', 'max', 'min'])
def test_gpu_watershed_4d_vs_oracle(ctx, agg):
    """4-D input end to end: normalize_channels, then the watershed on those values as given
    (prenormalized) -- against oracle.watershed_from_seeds on the 4-D array; also with a mask."""
    import torch
    shape, bs = (24, 64, 72), (12, 32, 36)
    x4 = np.stack([O.boundary_map(shape, origin=(0, 7 * c, 3 * c)) for c in range(3)])
    seeds = _seeds_from_ccl(ctx, np.ascontiguousarray(x4[0]), bs)
    sh = seeds.cpu().numpy().view(np.uint64)
    mask = (np.random.default_rng(5).random(shape) < 0.9).astype(np.uint8)
    for m in (None, mask):
        want = W.watershed_from_seeds(x4, sh, bs, m, 0, None, agg)
        xn = ctx.normalize_channels(torch.from_numpy(x4).cuda(), bs, agg)
        got, _ = ctx.watershed_from_seeds(xn, seeds, bs, None if m is None else torch.from_numpy(m).cuda(),
                                          prenormalized=True)
        np.testing.assert_array_equal(got.cpu().numpy().view(np.uint64), want)


def test_blocks_box():
    """The watershed job reads only the block-aligned bounding box of its blocks (blocks are
    independent: the box's own blocking is the volume's)."""
    from cluster_tools_amd.watershed.watershed_from_seeds import _blocks_box
    shape, bs = (20, 30, 45), (8, 16, 20)          # 3 x 2 x 3 blocks, edge blocks clipped
    _, box = _blocks_box(shape, bs, [4, 5])         # blocks (0, 1, 1) and (0, 1, 2)
    assert box == [(0, 8), (16, 30), (20, 45)]
    _, box = _blocks_box(shape, bs, list(range(18)))
    assert box == [(0, 20), (0, 30), (0, 45)]
    _, box = _blocks_box(shape, bs, [17])
    assert box == [(16, 20), (16, 30), (40, 45)]
