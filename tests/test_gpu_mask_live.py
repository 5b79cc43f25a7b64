"""Masked volumes whose blocks hold no mask voxel: the reference never reads such a block
(block_components.py:197-201 returns 0 before reading the input), and k_spec skips it
(k_mask_live's flags).  Against the oracle on the whole volume: fully masked blocks, blocks
whose only mask voxel sits anywhere in the block (the scan must find it), NaN / inf input inside
masked-out blocks, both modes and both single-volume schedules, and the z-slab path."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _volume(shape, bs, seed):
    rng = np.random.default_rng(seed)
    x = O.boundary_map(shape, origin=(seed, 2, 5))
    nb = [-(-a // b) for a, b in zip(shape, bs)]
    m = np.zeros(shape, np.uint8)
    kinds = rng.integers(0, 4, size=nb)                 # 0 empty, 1 one voxel, 2 partial, 3 full
    for bz in range(nb[0]):
        for by in range(nb[1]):
            for bx in range(nb[2]):
                sl = tuple(slice(i * b, min((i + 1) * b, s)) for i, b, s in zip((bz, by, bx), bs, shape))
                k = kinds[bz, by, bx]
                if k == 1:
                    ext = [s.stop - s.start for s in sl]
                    pos = tuple(s.start + int(rng.integers(0, e)) for s, e in zip(sl, ext))
                    m[pos] = 1
                elif k == 2:
                    m[sl] = (rng.random(tuple(s.stop - s.start for s in sl)) < 0.3).astype(np.uint8)
                elif k == 3:
                    m[sl] = 1
                else:
                    # input a masked-out block may hold: NaN / inf never matter there
                    x[sl][0, 0, 0] = np.nan
                    x[sl][-1, -1, -1] = np.inf
    return x, m


@pytest.mark.parametrize('mode', ['greater', 'less'])
@pytest.mark.parametrize('fast', ['1', '0'])
@pytest.mark.parametrize('shape,bs,seed', [((96, 200, 260), (32, 64, 64), 1), ((75, 130, 170), (25, 45, 63), 2),
                                           ((64, 256, 512), (64, 128, 256), 3)])
def test_mask_dead_blocks_vs_oracle(monkeypatch, ctx, mode, fast, shape, bs, seed):
    import torch
    monkeypatch.setenv('CC_FAST', fast)
    x, m = _volume(shape, bs, seed)
    ref = O.label_volume(x, bs, 0.5, mode, m, n_threads=8)
    lab, res = ctx.label_volume(torch.from_numpy(x).cuda(), bs, 0.5, mode, mask=torch.from_numpy(m).cuda())
    np.testing.assert_array_equal(lab.cpu().numpy().view(np.uint64), ref['labels'])
    assert res['n_labels'] == ref['n_labels']
    np.testing.assert_array_equal(ctx.lut(res['n_labels']), ref['lut'])
    np.testing.assert_array_equal(ctx.block_values(len(ref['values'])), ref['values'])


def test_mask_dead_blocks_sharded():
    """The z-slab path (both schedules) with fully masked blocks in every slab."""
    import torch
    from cluster_tools_amd import _lib
    from cluster_tools_amd.distributed import label_slabs_single_process, assemble_lut
    shape, bs = (96, 200, 260), (32, 64, 64)
    x, m = _volume(shape, bs, 7)
    ref = O.label_volume(x, bs, 0.5, 'greater', m, n_threads=8)
    for schedule in ('fast', 'sync'):
        ctxs = [_lib.Context(0) for _ in range(3)]
        try:
            lab, res, sums, luts = label_slabs_single_process(ctxs, torch.from_numpy(x).cuda(), bs, 0.5, 'greater',
                                                              mask=torch.from_numpy(m).cuda(), schedule=schedule)
            np.testing.assert_array_equal(lab.cpu().numpy().view(np.uint64), ref['labels'])
            np.testing.assert_array_equal(assemble_lut(luts, sums), ref['lut'])
        finally:
            for c in ctxs:
                c.close()


def test_misaligned_device_pointers_refused(ctx):
    """The kernels read rows with 16-B loads from the bases they are given: a contiguous view at an
    odd element offset is refused with an error (include/cc_mi355x.h), and the context stays usable."""
    import torch
    shape, bs = (16, 32, 32), (16, 32, 32)
    n = 16 * 32 * 32
    x = torch.zeros(n + 4, dtype=torch.float32, device='cuda')
    m = torch.ones(n + 1, dtype=torch.uint8, device='cuda')
    o = torch.empty(n + 1, dtype=torch.int64, device='cuda')
    for xi, mi, oi in ((x[1:n + 1], m[:n], o[:n]), (x[:n], m[1:], o[:n]), (x[:n], m[:n], o[1:])):
        with pytest.raises(RuntimeError, match='16-byte aligned'):
            ctx.label_volume(xi.view(shape), bs, 0.5, 'less', mask=mi.view(shape), out=oi.view(shape))
    lab, res = ctx.label_volume(x[:n].view(shape), bs, 0.5, 'less', mask=m[:n].view(shape))
    ref = O.label_volume(np.zeros(shape, np.float32), bs, 0.5, 'less', np.ones(shape, np.uint8), n_threads=1)
    np.testing.assert_array_equal(lab.cpu().numpy().view(np.uint64), ref['labels'])
    assert res['n_labels'] == ref['n_labels']


def test_slab_views_with_unaligned_rows_accepted(ctx):
    """A z-slab view keeps its rows' alignment (the rule the entries check, include/cc_mi355x.h):
    rows of 10 voxels need only 8-B (input), 2-B (mask) and 16-B (labels) bases, so views one
    plane into their storage are labelled, bit-exact against the oracle."""
    import torch
    full = (9, 6, 10)
    x = O.boundary_map(full, origin=(1, 2, 3))
    m = (np.random.default_rng(5).random(full) < 0.8).astype(np.uint8)
    xd, md = torch.from_numpy(x).cuda(), torch.from_numpy(m).cuda()
    od = torch.empty(full, dtype=torch.int64, device='cuda')
    for mode in ('greater', 'less'):
        lab, res = ctx.label_volume(xd[1:], (4, 6, 10), 0.5, mode, mask=md[1:], out=od[1:])
        ref = O.label_volume(np.ascontiguousarray(x[1:]), (4, 6, 10), 0.5, mode, np.ascontiguousarray(m[1:]),
                             n_threads=1)
        np.testing.assert_array_equal(lab.cpu().numpy().view(np.uint64), ref['labels'])
        assert res['n_labels'] == ref['n_labels']
