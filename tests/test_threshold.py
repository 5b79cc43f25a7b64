"""Threshold task (reference cluster_tools/thresholded_components/threshold.py): the numpy
oracle against the golden vectors made by the reference's own `threshold` job
(tests/golden/make_golden_threshold.py), and the HIP path (cc_threshold) against both, through
the ctx API and through the ThresholdLocal task on N5."""
import glob
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, load_golden
from oracle import oracle as O

CASES = sorted(os.path.basename(p)[len('threshold_'):-len('.npz')]
               for p in glob.glob(os.path.join(GOLDEN, 'threshold_*.npz')))


def _case(name):
    z = np.load(os.path.join(GOLDEN, 'threshold_%s.npz' % name))
    return (load_golden(name)['input'], tuple(int(v) for v in z['block_shape']), float(z['threshold']),
            str(z['mode']), z['expected'])


def test_cases_present():
    assert len(CASES) >= 12


@pytest.mark.parametrize('name', CASES)
def test_oracle_matches_reference(name):
    x, bs, t, mode, exp = _case(name)
    np.testing.assert_array_equal(O.threshold_volume(x, bs, t, mode), exp)


@pytest.mark.gpu
@pytest.mark.parametrize('name', CASES)
def test_gpu_matches_reference(ctx, name):
    import torch
    x, bs, t, mode, exp = _case(name)
    got = ctx.threshold(torch.from_numpy(x).cuda(), bs, t, mode).cpu().numpy()
    np.testing.assert_array_equal(got, exp)


@pytest.mark.gpu
@pytest.mark.parametrize('shape,bs,mode', [((96, 200, 256), (64, 100, 128), 'greater'),
                                           ((70, 130, 203), (32, 64, 50), 'less'),
                                           ((64, 128, 128), (64, 128, 128), 'equal'),
                                           # four full tiles of one block per workgroup (16-B stores)
                                           ((48, 96, 512), (32, 64, 256), 'greater'),
                                           ((48, 96, 768), (48, 96, 384), 'less')])
def test_gpu_matches_oracle_larger(ctx, shape, bs, mode):
    """Full and ragged tiles (float4 and scalar paths), unaligned X, one-block volumes."""
    import torch
    x = O.boundary_map(shape, origin=(5, 3, 1))
    t = 0.5 if mode != 'equal' else 0.0
    got = ctx.threshold(torch.from_numpy(x).cuda(), bs, t, mode).cpu().numpy()
    np.testing.assert_array_equal(got, O.threshold_volume(x, bs, t, mode))


@pytest.mark.gpu
def test_threshold_task_n5(tmp_path):
    from cluster_tools_amd import luigi_compat as luigi, n5
    from cluster_tools_amd.cluster_tasks import BaseClusterTask
    from cluster_tools_amd.thresholded_components.threshold import ThresholdLocal
    name = 'norm_edge_greater'
    x, bs, t, mode, exp = _case(name)
    data = str(tmp_path / 'data.n5')
    with n5.open_file(data) as f:
        f.create_dataset('raw', data=x, chunks=(4, 8, 8), compression='gzip')
    cfg = str(tmp_path / 'config')
    os.makedirs(cfg)
    g = BaseClusterTask.default_global_config()
    g['block_shape'] = list(bs)
    with open(os.path.join(cfg, 'global.config'), 'w') as f:
        json.dump(g, f)
    task = ThresholdLocal(tmp_folder=str(tmp_path / 'tmp'), config_dir=cfg, max_jobs=2, input_path=data,
                          input_key='raw', output_path=data, output_key='thr', threshold=t, threshold_mode=mode)
    assert luigi.build([task], local_scheduler=True)
    with n5.open_file(data, 'r') as f:
        ds = f['thr']
        assert ds.dtype == np.uint8
        assert tuple(ds.chunks) == tuple(max(1, min(b // 2, s)) for b, s in zip(bs, x.shape))
        np.testing.assert_array_equal(ds[:], exp)
    assert (tmp_path / 'tmp' / 'threshold.log').exists()


@pytest.mark.gpu
@pytest.mark.parametrize('variant', ['spec', 'no_guess', 'two_pass'])
@pytest.mark.parametrize('mode,thr', [('greater', 0.5), ('less', 0.37), ('equal', 0.5)])
def test_gpu_speculative_threshold_corrected(ctx, monkeypatch, variant, mode, thr):
    """The one-read Threshold (k_thr_spec: guessed interval, exact statistics + TB, k_thr_fix of
    the listed tiles) on inputs whose guess misses: continuous (dithered) data and block extremes
    off the sampled rows; against the oracle, and the no-guess / two-pass variants."""
    import torch
    if variant == 'no_guess':
        monkeypatch.setenv('CC_SPEC', '0')
    elif variant == 'two_pass':
        monkeypatch.setenv('CC_THRESHOLD_TWO_PASS', '1')
    rng = np.random.default_rng(3)
    q = (rng.integers(0, 17, (64, 128, 192)) / np.float32(16)).astype(np.float32)
    q[1, 1, 5] = -1.0                      # outliers off the sampled rows (z = 8 mod 16, y = 16 mod 32)
    q[33, 70, 100] = 3.0
    q2 = (rng.integers(0, 17, (64, 128, 512)) / np.float32(16)).astype(np.float32)
    q2[2, 3, 300] = -1.0                   # outliers off the sampled rows, in four-tile workgroups
    q2[40, 99, 17] = 3.0
    for x, bs in [(O.boundary_map((96, 200, 256), origin=(5, 3, 1), dither=True), (32, 100, 128)),
                  (O.boundary_map((64, 128, 512), origin=(5, 3, 1), dither=True), (32, 64, 256)),
                  (q, (32, 64, 96)), (q, (64, 128, 192)), (q2, (32, 128, 256))]:
        got = ctx.threshold(torch.from_numpy(x).cuda(), bs, thr, mode).cpu().numpy()
        np.testing.assert_array_equal(got, O.threshold_volume(x, bs, thr, mode))
