"""Segmentation evaluation (reference EvaluationWorkflow: node_labels/block_node_labels.py:133-166
overlaps + evaluation/measures.py:81-162 measures).  CPU: the numpy oracle on hand-computed
cases and the block-skip / ignore-label rules.  GPU: cc_evaluate against the oracle -- the
contingency table bit-exact, the measures to 1e-9 -- on ragged shapes and block grids, table
growth, and the partition-equality property at volume scale.

The measure formulas restate elf (absent here): parity of those formulas is unpinned, see
oracle/evaluation.py."""
import numpy as np
import pytest

from oracle import evaluation as E

RTOL = 1e-9


def _vol(a):
    return np.asarray(a, dtype=np.uint64).reshape(1, 1, -1)


def test_oracle_hand_case():
    seg, gt = _vol([1, 1, 2, 2]), _vol([1, 1, 1, 1])
    m, ov = E.measures(seg, gt, (1, 1, 4), ignore_label=None)
    assert ov == {(1, 1): 2, (2, 1): 2}
    assert m['n_points'] == 4 and m['n_pairs'] == 2
    assert m['vi_split'] == pytest.approx(1.0) and m['vi_merge'] == pytest.approx(0.0, abs=1e-15)
    assert m['adapted_rand_error'] == pytest.approx(1.0 / 3.0)
    assert m['rand_index'] == pytest.approx(0.5)


def test_oracle_identical_partitions():
    rng = np.random.default_rng(3)
    seg = rng.integers(1, 20, size=(6, 7, 9)).astype(np.uint64)
    perm = rng.permutation(np.arange(100, 120, dtype=np.uint64))
    gt = perm[seg.astype(np.int64) - 1]
    m, _ = E.measures(seg, gt, (4, 4, 4), ignore_label=None)
    assert abs(m['vi_split']) < 1e-12 and abs(m['vi_merge']) < 1e-12
    assert m['rand_index'] == pytest.approx(1.0) and abs(m['adapted_rand_error']) < 1e-12


def test_oracle_block_skip_and_ignore():
    # block 0 (x 0..1): seg all zero -> skipped (block_node_labels.py:141); block 1 keeps its
    # seg-0 voxel; gt == 0 voxels are ignored
    seg, gt = _vol([0, 0, 0, 5]), _vol([3, 4, 7, 0])
    _, ov = E.measures(seg, gt, (1, 1, 2), ignore_label=0)
    assert ov == {(0, 7): 1}
    _, ov = E.measures(seg, gt, (1, 1, 2), ignore_label=None)
    assert ov == {(0, 7): 1, (5, 0): 1}
    _, ov = E.measures(seg, gt, (1, 1, 4), ignore_label=0)
    assert ov == {(0, 3): 1, (0, 4): 1, (0, 7): 1}


def _random_case(rng, shape, n_seg, n_gt, zero_frac, ignore_frac):
    seg = rng.integers(1, n_seg + 1, size=shape).astype(np.uint64)
    seg[rng.random(shape) < zero_frac] = 0
    # whole zero slabs so that some blocks hold no seg at all
    seg[: max(1, shape[0] // 3)] = 0
    seg[:, :, : shape[2] // 2][rng.random(seg[:, :, : shape[2] // 2].shape) < 0.5] = 0
    gt = rng.integers(1, n_gt + 1, size=shape).astype(np.uint64)
    gt[rng.random(shape) < ignore_frac] = 0
    return seg, gt


CASES = [
    ((3, 5, 7), (2, 2, 3), 4, 3, 0.3, 0.2),
    ((9, 17, 33), (4, 8, 8), 6, 5, 0.2, 0.1),
    ((16, 40, 72), (16, 16, 16), 30, 12, 0.1, 0.05),
    ((5, 64, 130), (5, 64, 130), 500, 300, 0.0, 0.0),
    ((20, 31, 45), (7, 10, 13), 1, 1, 0.5, 0.3),
]


@pytest.mark.gpu
@pytest.mark.parametrize('case', range(len(CASES)))
@pytest.mark.parametrize('ignore', [0, None])
def test_gpu_evaluate_matches_oracle(ctx, case, ignore):
    import torch
    shape, bs, ns, ng, zf, igf = CASES[case]
    rng = np.random.default_rng(100 + case)
    seg, gt = _random_case(rng, shape, ns, ng, zf, igf)
    want, ov = E.measures(seg, gt, bs, ignore_label=ignore)
    dseg = torch.from_numpy(seg.view(np.int64)).cuda()
    dgt = torch.from_numpy(gt.view(np.int64)).cuda()
    got = ctx.evaluate(dseg, dgt, bs, ignore_label=ignore)
    for k in ('n_points', 'n_pairs', 'n_seg_ids', 'n_gt_ids'):
        assert got[k] == want[k], k
    s, g, c = ctx.overlaps()
    assert {(int(a), int(b)): int(n) for a, b, n in zip(s, g, c)} == ov
    if want['n_points']:
        for k in ('vi_split', 'vi_merge', 'adapted_rand_error', 'rand_index'):
            assert got[k] == pytest.approx(want[k], rel=RTOL, abs=1e-12), k


@pytest.mark.gpu
def test_gpu_evaluate_empty_and_errors(ctx):
    import torch
    z = torch.zeros((4, 8, 8), dtype=torch.int64, device='cuda')
    got = ctx.evaluate(z, z, (2, 4, 4))
    assert got['n_points'] == 0 and got['n_pairs'] == 0



@pytest.mark.gpu
@pytest.mark.parametrize('ignore', [0, 5, None])
def test_gpu_evaluate_sparse_64bit_ids(ctx, ignore):
    """Ids beyond the device key packing (seg >= 2^31, gt >= 2^32 - 1, up to 2^64 - 2) are
    relabelled consecutively on the device first: the measures equal those of the small-id
    volumes, and overlaps() reports the caller's ids."""
    import torch
    rng = np.random.default_rng(21)
    shape, bs = (9, 17, 33), (4, 8, 8)
    seg, gt = _random_case(rng, shape, 6, 5, 0.2, 0.1)
    want, ov = E.measures(seg, gt, bs, ignore_label=ignore)

    def sparse(a):     # order-preserving, 0 -> 0, ignore label kept
        b = a.astype(np.uint64) * np.uint64(0x0123456789ABC) + np.uint64(1 << 62)
        b[a == 0] = 0
        if ignore:
            b[a == ignore] = ignore
        return b
    s64, g64 = sparse(seg), sparse(gt)
    got = ctx.evaluate(torch.from_numpy(s64.view(np.int64)).cuda(), torch.from_numpy(g64.view(np.int64)).cuda(),
                       bs, ignore_label=ignore)
    for k in ('n_points', 'n_pairs', 'n_seg_ids', 'n_gt_ids'):
        assert got[k] == want[k], k
    for k in ('vi_split', 'vi_merge', 'adapted_rand_error', 'rand_index'):
        assert got[k] == pytest.approx(want[k], rel=RTOL, abs=1e-12), k
    _, ov64 = E.measures(s64, g64, bs, ignore_label=ignore)
    sa, gb, cnt = ctx.overlaps()
    assert {(int(a), int(b)): int(n) for a, b, n in zip(sa, gb, cnt)} == ov64


@pytest.mark.gpu
def test_gpu_evaluate_table_growth(ctx):
    """~1M distinct pairs: more than the first table (2^20 entries, kept at most half full) holds."""
    import torch
    rng = np.random.default_rng(7)
    shape = (64, 128, 128)
    seg = rng.integers(1, 1 << 20, size=shape).astype(np.uint64)
    gt = rng.integers(1, 1 << 20, size=shape).astype(np.uint64)
    want, ov = E.measures(seg, gt, (32, 64, 64), ignore_label=0)
    got = ctx.evaluate(torch.from_numpy(seg.view(np.int64)).cuda(),
                       torch.from_numpy(gt.view(np.int64)).cuda(), (32, 64, 64))
    assert got['n_pairs'] == want['n_pairs'] == len(ov)
    for k in ('vi_split', 'vi_merge', 'adapted_rand_error', 'rand_index'):
        assert got[k] == pytest.approx(want[k], rel=RTOL, abs=1e-12), k


@pytest.mark.gpu
def test_gpu_evaluate_cc_labels_at_scale(ctx):
    """Property at volume scale: the CCL output against a permuted relabelling of itself is the
    same partition (VI 0, RI 1, ARE 0); against the 'less' labelling with ignore label 0 the
    counted voxels are the 'greater' background (n_points = voxels with gt != 0)."""
    import torch
    shape, bs = (256, 1024, 1024), (64, 512, 512)
    inp = ctx.generate_boundary_map(shape)
    seg, r = ctx.label_volume(inp, bs, 0.5, 'greater')
    perm = torch.randperm(int(r['n_labels']) + 7, device='cuda')[: int(r['n_labels'])] + 1
    perm[0] = 0
    gt = perm[seg]
    got = ctx.evaluate(seg, gt, bs, ignore_label=None)
    assert got['n_points'] == seg.numel()
    assert abs(got['vi_split']) < 1e-9 and abs(got['vi_merge']) < 1e-9
    assert abs(got['rand_index'] - 1.0) < 1e-12 and abs(got['adapted_rand_error']) < 1e-12
    assert got['n_pairs'] == got['n_seg_ids'] == got['n_gt_ids']
    gt2, _ = ctx.label_volume(inp, bs, 0.5, 'less')
    got = ctx.evaluate(seg, gt2, bs, ignore_label=0)
    assert got['n_points'] == int((gt2 != 0).sum())   # every block holds seg (membranes)
    # 'less' foreground is exactly the 'greater' background: every counted voxel has seg 0, so
    # seg splits nothing and merges every gt object
    assert got['n_seg_ids'] == 1 and got['n_pairs'] == got['n_gt_ids']
    assert abs(got['vi_split']) < 1e-9 and got['vi_merge'] > 1.0 and 0.0 < got['rand_index'] < 1.0


@pytest.mark.gpu
def test_gpu_ccl_partition_deterministic_c3(ctx):
    """Regression: at C3 'less' (150k components) a path-compression race in the tile CCL
    (cc_kernels.hip tile_ccl phase 3) moved a handful of 7-60 voxel pieces to another component
    of their tile in ~8 of 256 blocks per run.  Two runs must give the same partition: the
    contingency table of run a against run b is a bijection (pairs == ids on both sides)."""
    shape, bs = (1024, 2048, 2048), (64, 512, 512)
    inp = ctx.generate_boundary_map(shape)
    a, ra = ctx.label_volume(inp, bs, 0.5, 'less')
    for _ in range(2):
        b, rb = ctx.label_volume(inp, bs, 0.5, 'less')
        r = ctx.evaluate(a, b, bs, ignore_label=None)
        assert ra == rb
        assert r['n_pairs'] == r['n_seg_ids'] == r['n_gt_ids'] == ra['n_components'] + 1
        del b


@pytest.mark.gpu
def test_gpu_evaluation_workflow(tmp_path):
    """EvaluationWorkflow through the task API on N5 (evaluation_workflow.py:46-84 surface):
    the output JSON carries the reference's four keys, equal to the oracle's measures."""
    import json
    import os
    from cluster_tools_amd import luigi_compat as luigi, n5
    from cluster_tools_amd.cluster_tasks import BaseClusterTask
    from cluster_tools_amd.evaluation import EvaluationWorkflow
    rng = np.random.default_rng(11)
    shape, bs = (12, 40, 56), [6, 16, 32]
    seg, gt = _random_case(rng, shape, 9, 7, 0.2, 0.1)
    data = str(tmp_path / 'data.n5')
    with n5.open_file(data) as f:
        f.create_dataset('seg', data=seg, chunks=(6, 16, 16), compression='gzip')
        f.create_dataset('gt', data=gt, chunks=(6, 16, 16), compression='gzip')
    cfg = str(tmp_path / 'config')
    os.makedirs(cfg)
    g = BaseClusterTask.default_global_config()
    g['block_shape'] = bs
    with open(os.path.join(cfg, 'global.config'), 'w') as f:
        json.dump(g, f)
    out = str(tmp_path / 'scores.json')
    t = EvaluationWorkflow(tmp_folder=str(tmp_path / 'tmp'), config_dir=cfg, target='local', max_jobs=1,
                           seg_path=data, seg_key='seg', gt_path=data, gt_key='gt', output_path=out)
    assert luigi.build([t], local_scheduler=True)
    with open(out) as f:
        got = json.load(f)
    want, _ = E.measures(seg, gt, bs, ignore_label=0)
    assert set(got) == {'vi-split', 'vi-merge', 'adapted-rand-error', 'rand-index'}
    for k, w in (('vi-split', 'vi_split'), ('vi-merge', 'vi_merge'),
                 ('adapted-rand-error', 'adapted_rand_error'), ('rand-index', 'rand_index')):
        assert got[k] == pytest.approx(want[w], rel=RTOL, abs=1e-12), k
