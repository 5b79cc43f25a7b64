"""Multi-channel input (`channel` of BlockComponents / Threshold / the workflow; reference
block_components.py:150-159, threshold.py:139-148): the numpy restatement (oracle.channel_mean)
against the golden vectors made by the reference's own jobs (tests/golden/make_golden_channel.py),
then the device mean (cc_channel_mean) bit-exact against it and the labelling / threshold /
workflow on top of it against the reference's artefacts."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, load_golden
from oracle import oracle as O

with open(os.path.join(GOLDEN, 'index_channel.json')) as _f:
    INDEX = json.load(_f)
CASES = sorted(INDEX)


def _case(name):
    return load_golden('channel_' + name), INDEX[name]


def _chans(d):
    return [int(c) for c in d['channel']]


@pytest.mark.parametrize('name', CASES)
def test_oracle_matches_reference(name):
    d, meta = _case(name)
    x = O.channel_mean(d['input'], meta['channel'])
    bs, thr = meta['block_shape'], float(d['threshold'])
    np.testing.assert_array_equal(O.threshold_volume(x, bs, thr, meta['mode']), d['thr_expected'])
    r = O.label_volume(x, bs, thr, meta['mode'], d.get('mask'), n_threads=3, want_local=True)
    np.testing.assert_array_equal(r['local'], d['local_labels'].astype(np.uint64))
    np.testing.assert_array_equal(r['values'], d['block_values'])
    np.testing.assert_array_equal(r['offsets'], d['offsets'])
    np.testing.assert_array_equal(O.canon(r['labels']), d['labels_canon'])
    np.testing.assert_array_equal(O.canon(r['lut']), d['lut_canon'])
    assert r['max_id'] == int(d['max_id'])


def test_summation_order_is_pinned():
    """The float32 cases are order-sensitive: summing the same channels in another order gives
    other float32 means, so the goldens pin the reference's left-to-right accumulation."""
    d, meta = _case('f32_rev')
    ch = _chans(d)
    want = O.channel_mean(d['input'], ch)
    other = O.channel_mean(d['input'], ch[::-1])
    assert np.count_nonzero(want != other) > 0
    assert want.dtype == np.float32


def test_channel_list_parsing():
    from cluster_tools_amd.thresholded_components.block_components import channel_list
    assert channel_list(2) == [2]
    assert channel_list([0, 2, 0]) == [0, 2, 0]
    assert channel_list((1,)) == [1]
    assert channel_list('[3, 1]') == [3, 1]
    assert channel_list(np.int64(4)) == [4]


@pytest.mark.gpu
@pytest.mark.parametrize('name', CASES)
def test_gpu_mean_and_labels_match_reference(ctx, name):
    import torch
    d, meta = _case(name)
    want = O.channel_mean(d['input'], meta['channel'])
    x = ctx.channel_mean(d['input'], meta['channel'])                # numpy upload (raw bytes)
    np.testing.assert_array_equal(x.cpu().numpy(), want)
    if d['input'].dtype in (np.float32, np.float64, np.int64, np.int16, np.int32, np.uint8):
        x2 = ctx.channel_mean(torch.from_numpy(d['input']).cuda(), meta['channel'])   # torch tensor
        np.testing.assert_array_equal(x2.cpu().numpy(), want)
    bs, thr = meta['block_shape'], float(d['threshold'])
    np.testing.assert_array_equal(ctx.threshold(x, bs, thr, meta['mode']).cpu().numpy(), d['thr_expected'])
    m = torch.from_numpy(d['mask']).cuda() if 'mask' in d else None
    lab, res = ctx.label_volume(x, bs, thr, meta['mode'], m)
    np.testing.assert_array_equal(O.canon(lab.cpu().numpy()), d['labels_canon'])
    np.testing.assert_array_equal(ctx.block_values(len(d['block_values'])), d['block_values'])
    np.testing.assert_array_equal(O.canon(ctx.lut(res['n_labels'])), d['lut_canon'])
    assert res['max_id'] == int(d['max_id'])
    local, values = ctx.block_components(x, bs, thr, meta['mode'], m)
    np.testing.assert_array_equal(local.cpu().numpy().view(np.uint64), d['local_labels'].astype(np.uint64))


@pytest.mark.gpu
@pytest.mark.parametrize('dtype', ['float32', 'float64', 'uint8', 'int8', 'uint16', 'int16', 'uint32', 'int32',
                                   'uint64', 'int64'])
@pytest.mark.parametrize('shape', [(3, 16, 32, 64), (4, 7, 13, 29)])      # vector path / scalar tail
def test_gpu_mean_dtypes_vs_oracle(ctx, dtype, shape):
    rng = np.random.default_rng(7)
    dt = np.dtype(dtype)
    if dt.kind == 'f':
        a = (rng.standard_normal(shape) * np.array([1.0, 1e4, 1e-3, 7.0][:shape[0]]).reshape(-1, 1, 1, 1)).astype(dt)
    else:
        info = np.iinfo(dt)
        a = rng.integers(info.min, info.max, size=shape, dtype=dt, endpoint=True)
    for chans in ([1], [0, 2], [2, 0, 1, 2]):
        np.testing.assert_array_equal(ctx.channel_mean(a, chans).cpu().numpy(), O.channel_mean(a, chans))


@pytest.mark.gpu
def test_gpu_mean_rejects_bad_channels(ctx):
    a = np.zeros((2, 4, 4, 4), np.float32)
    with pytest.raises(RuntimeError):
        ctx.channel_mean(a, [2])
    with pytest.raises(RuntimeError):
        ctx.channel_mean(a, list(range(65)))


@pytest.mark.gpu
@pytest.mark.parametrize('name,fused', [('bmap3_less_mask', True), ('f32_pair', True), ('u8_pair', True),
                                        ('f32_int', False)])
def test_workflow_channel_n5(tmp_path, name, fused):
    """ThresholdedComponentsWorkflow on a 4-D N5 dataset with `channel` (fused job; fused=False:
    the stage tasks one by one) and the Threshold task on the same dataset.  (Cases with even
    block shapes: the Write task requires block_shape % chunks == 0, write.py:54, as upstream.)"""
    from cluster_tools_amd import luigi_compat as luigi, n5
    from cluster_tools_amd.cluster_tasks import BaseClusterTask
    from cluster_tools_amd.thresholded_components import ThresholdedComponentsWorkflow
    from cluster_tools_amd.thresholded_components.threshold import ThresholdLocal
    d, meta = _case(name)
    data = str(tmp_path / 'data.n5')
    with n5.open_file(data) as f:
        f.create_dataset('raw', data=d['input'], chunks=(1, 8, 16, 16), compression='gzip')
        if 'mask' in d:
            f.create_dataset('mask', data=d['mask'], chunks=(8, 16, 16), compression='gzip')
    cfg = str(tmp_path / 'config')
    os.makedirs(cfg)
    g = BaseClusterTask.default_global_config()
    g['block_shape'] = list(meta['block_shape'])
    with open(os.path.join(cfg, 'global.config'), 'w') as f:
        json.dump(g, f)
    kw = dict(mask_path=data, mask_key='mask') if 'mask' in d else {}
    t = ThresholdedComponentsWorkflow(tmp_folder=str(tmp_path / 'tmp'), config_dir=cfg, target='local', max_jobs=2,
                                      input_path=data, input_key='raw', output_path=data, output_key='seg',
                                      assignment_key='assignments', threshold=float(d['threshold']),
                                      threshold_mode=meta['mode'], channel=meta['channel'], fused=fused, **kw)
    assert luigi.build([t], local_scheduler=True)
    th = ThresholdLocal(tmp_folder=str(tmp_path / 'tmp_thr'), config_dir=cfg, max_jobs=2, input_path=data,
                        input_key='raw', output_path=data, output_key='thr', threshold=float(d['threshold']),
                        threshold_mode=meta['mode'], channel=meta['channel'])
    assert luigi.build([th], local_scheduler=True)
    with n5.open_file(data, 'r') as f:
        np.testing.assert_array_equal(O.canon(f['seg'][:]), d['labels_canon'])
        np.testing.assert_array_equal(O.canon(f['assignments'][:]), d['lut_canon'])
        assert f['seg'].attrs['maxId'] == int(d['max_id'])
        np.testing.assert_array_equal(f['thr'][:], d['thr_expected'])
