"""Consecutive relabelling (reference RelabelWorkflow: relabel/find_uniques.py,
find_labeling.py:84-120, write): cc_relabel_consecutive against the numpy oracle -- volume and
assignment table bit-exact -- with and without id 0, sparse 64-bit ids, in place, table
growth, and idempotence at C3 scale."""
import numpy as np
import pytest

from oracle import relabel as R


def test_oracle_start_label():
    out, a = R.relabel_consecutive(np.array([[[5, 0, 9, 5]]], dtype=np.uint64))
    assert out.tolist() == [[[1, 0, 2, 1]]] and a.tolist() == [[0, 0], [5, 1], [9, 2]]
    out, a = R.relabel_consecutive(np.array([[[7, 3, 3]]], dtype=np.uint64))
    assert out.tolist() == [[[2, 1, 1]]] and a.tolist() == [[3, 1], [7, 2]]


@pytest.mark.gpu
@pytest.mark.parametrize('case', ['zeros_runs', 'no_zero_sparse', 'many_ids', 'tiny', 'runs_big', 'unaligned_odd'])
def test_gpu_relabel_matches_oracle(ctx, case):
    import torch
    rng = np.random.default_rng(5)
    if case == 'zeros_runs':
        lab = np.repeat(rng.integers(0, 50, size=(20, 30, 8)), 8, axis=2).astype(np.uint64) * np.uint64(1000)
    elif case == 'no_zero_sparse':
        lab = rng.integers(1, 1 << 62, size=(7, 33, 65), dtype=np.int64).astype(np.uint64)
        lab[:, :, :30] = lab[0, 0, 0]
    elif case == 'many_ids':       # > the first id set (2^16 slots, with the small cap_hint below)
        lab = rng.integers(0, 1 << 40, size=(16, 128, 128), dtype=np.int64).astype(np.uint64)
    elif case == 'runs_big':       # several workgroup ranges, runs crossing lanes and ranges
        lab = np.repeat(rng.integers(0, 3000, size=(40, 64, 32)), 37, axis=2).astype(np.uint64)
    elif case == 'unaligned_odd':  # 8-B but not 16-B aligned, odd length: the one-id-per-lane path
        lab = np.repeat(rng.integers(0, 900, size=(9, 31, 29)), 3, axis=2).astype(np.uint64)
    else:
        lab = np.array([[[3]]], dtype=np.uint64)
    want, wa = R.relabel_consecutive(lab)
    d = torch.from_numpy(lab.view(np.int64)).cuda()
    if case == 'unaligned_odd':
        buf = torch.empty(d.numel() + 1, dtype=torch.int64, device='cuda')
        buf[1:] = d.reshape(-1)
        d = buf[1:].view(d.shape)
        assert d.data_ptr() % 16 == 8
    # many_ids: a small capacity hint, so the device id set (2^16 slots) grows and the host table
    # is too small for the first call (the second call has the exact size)
    out, table = ctx.relabel_consecutive(d, cap_hint=1024 if case == 'many_ids' else 1 << 20)
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint64), want)
    np.testing.assert_array_equal(table, wa)
    out2, table2 = ctx.relabel_consecutive(d, out=d)     # in place
    np.testing.assert_array_equal(d.cpu().numpy().view(np.uint64), want)
    np.testing.assert_array_equal(table2, wa)


@pytest.mark.gpu
def test_gpu_relabel_c3_scale(ctx):
    """C3 'less' labels: consecutive ids 1..n_components (0 kept), relabelling is idempotent,
    and the partition is unchanged (device contingency table is a bijection)."""
    shape, bs = (1024, 2048, 2048), (64, 512, 512)
    x = ctx.generate_boundary_map(shape)
    lab, r = ctx.label_volume(x, bs, 0.5, 'less')
    del x
    out, table = ctx.relabel_consecutive(lab)
    n = r['n_components'] + 1
    assert table.shape == (n, 2) and table[0, 0] == 0 and int(table[-1, 1]) == n - 1
    assert int(out.max()) == n - 1
    again, t2 = ctx.relabel_consecutive(out)
    assert bool((again == out).all()) and np.array_equal(t2[:, 0], t2[:, 1])
    e = ctx.evaluate(lab, out, bs, ignore_label=None)
    assert e['n_pairs'] == e['n_seg_ids'] == e['n_gt_ids'] == n
