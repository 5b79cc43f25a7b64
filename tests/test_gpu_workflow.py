"""ThresholdedComponentsWorkflow end to end through the task API on N5 (the drop-in path), and
the five stage tasks run one by one (like test/thresholded_components/thresholded_components.py
of the reference), against the golden vectors made by the reference's own job functions."""
import json
import os

import numpy as np
import pytest

from conftest import load_golden
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _build(tasks, tmp):
    """luigi.build, printing the jobs' error logs when it fails (the job processes' tracebacks)."""
    import glob
    from cluster_tools_amd import luigi_compat as luigi
    ok = luigi.build(tasks, local_scheduler=True)
    if not ok:
        for p in sorted(glob.glob(os.path.join(str(tmp), 'error_logs', '*.err'))):
            txt = open(p).read()
            if txt.strip():
                print('==== %s\n%s' % (p, txt[-4000:]))
    return ok


def _setup(tmp_path, name, block_shape):
    from cluster_tools_amd import n5
    from cluster_tools_amd.cluster_tasks import BaseClusterTask
    d = load_golden(name)
    data = str(tmp_path / 'data.n5')
    with n5.open_file(data) as f:
        f.create_dataset('volumes/boundaries', data=d['input'], chunks=(8, 32, 32), compression='gzip')
        if 'mask' in d:
            f.create_dataset('volumes/mask', data=d['mask'], chunks=(8, 32, 32), compression='gzip')
    cfg = str(tmp_path / 'config')
    os.makedirs(cfg)
    g = BaseClusterTask.default_global_config()
    g['block_shape'] = list(block_shape)
    with open(os.path.join(cfg, 'global.config'), 'w') as f:
        json.dump(g, f)
    return d, data, cfg


@pytest.mark.parametrize('name', ['bmap_greater', 'bmap_less', 'bmap_mask', 'noise_tiny_blocks'])
def test_workflow_fused(tmp_path, name):
    from cluster_tools_amd import luigi_compat as luigi, n5
    from cluster_tools_amd.thresholded_components import ThresholdedComponentsWorkflow
    from conftest import golden_index
    meta = golden_index()[name]
    d, data, cfg = _setup(tmp_path, name, meta['block_shape'])
    kw = {}
    if 'mask' in d:
        kw = dict(mask_path=data, mask_key='volumes/mask')
    t = ThresholdedComponentsWorkflow(tmp_folder=str(tmp_path / 'tmp'), config_dir=cfg, target='local', max_jobs=4,
                                      input_path=data, input_key='volumes/boundaries', output_path=data,
                                      output_key='data', assignment_key='assignments',
                                      threshold=float(d['threshold']), threshold_mode=meta['mode'], **kw)
    assert _build([t], tmp_path / 'tmp')
    with n5.open_file(data, 'r') as f:
        seg = f['data'][:]
        lut = f['assignments'][:]
        max_id = f['data'].attrs['maxId']
    np.testing.assert_array_equal(O.canon(seg), d['labels_canon'])
    np.testing.assert_array_equal(O.canon(lut), d['lut_canon'])
    assert max_id == int(d['max_id'])
    off = json.load(open(str(tmp_path / 'tmp' / 'cc_offsets.json')))
    np.testing.assert_array_equal(np.array(off['offsets'], dtype=np.uint64), d['offsets'])
    np.testing.assert_array_equal(off['empty_blocks'], d['empty_blocks'])
    assert off['n_labels'] == int(d['n_labels'])
    for task in ('block_components', 'merge_offsets', 'block_faces', 'merge_assignments',
                 'write_thresholded_components'):
        assert (tmp_path / 'tmp' / (task + '.log')).exists(), task


def test_stage_by_stage(tmp_path):
    """Each stage task on its own (fused=False): BlockComponents writes the reference's
    block-local labels, BlockFaces / MergeAssignments / Write do the real work."""
    from cluster_tools_amd import luigi_compat as luigi, n5
    from cluster_tools_amd.cluster_tasks import DummyTask
    from cluster_tools_amd.thresholded_components.block_components import BlockComponentsLocal
    from cluster_tools_amd.thresholded_components.merge_offsets import MergeOffsetsLocal
    from cluster_tools_amd.thresholded_components.block_faces import BlockFacesLocal
    from cluster_tools_amd.thresholded_components.merge_assignments import MergeAssignmentsLocal
    from cluster_tools_amd.write import WriteLocal
    name = 'bmap_less'
    bs = (16, 32, 32)
    d, data, cfg = _setup(tmp_path, name, bs)
    tmp = str(tmp_path / 'tmp')
    common = dict(tmp_folder=tmp, config_dir=cfg, max_jobs=4)
    t1 = BlockComponentsLocal(input_path=data, input_key='volumes/boundaries', output_path=data, output_key='data',
                              threshold=0.5, threshold_mode='less', dependency=DummyTask(), **common)
    assert _build([t1], tmp)
    with n5.open_file(data, 'r') as f:
        np.testing.assert_array_equal(f['data'][:], d['local_labels'].astype(np.uint64))
    off_path = os.path.join(tmp, 'cc_offsets.json')
    shape = list(d['input'].shape)
    t2 = MergeOffsetsLocal(shape=shape, save_path=off_path, dependency=t1, **common)
    t3 = BlockFacesLocal(input_path=data, input_key='data', offsets_path=off_path, dependency=t2, **common)
    t4 = MergeAssignmentsLocal(output_path=data, output_key='assignments', shape=shape, offset_path=off_path,
                               dependency=t3, **common)
    t5 = WriteLocal(input_path=data, input_key='data', output_path=data, output_key='data',
                    assignment_path=data, assignment_key='assignments', identifier='thresholded_components',
                    offset_path=off_path, dependency=t4, **common)
    assert _build([t5], tmp)
    np.testing.assert_array_equal(np.load(os.path.join(tmp, 'cc_assignments_0.npy')), d['pairs'])
    with n5.open_file(data, 'r') as f:
        np.testing.assert_array_equal(O.canon(f['data'][:]), d['labels_canon'])
        np.testing.assert_array_equal(O.canon(f['assignments'][:]), d['lut_canon'])
        assert f['data'].attrs['maxId'] == int(d['max_id'])


def _write_task_config(cfg, name, values):
    with open(os.path.join(cfg, name + '.config'), 'w') as f:
        json.dump(values, f)


@pytest.mark.parametrize('gpus', [1, 2])
@pytest.mark.parametrize('name', ['bmap_quirk', 'bmap_greater', 'bmap_less'])
def test_workflow_empty_job_emulation(tmp_path, name, gpus):
    """merge_assignments config 'reference_empty_job_quirk' with the golden run's face-job count as
    max_jobs: the fused job reproduces the reference's output (identity LUT for bmap_quirk)."""
    from cluster_tools_amd import n5
    from cluster_tools_amd.thresholded_components import ThresholdedComponentsWorkflow
    from cluster_tools_amd.thresholded_components.merge_assignments import MergeAssignmentsLocal
    from conftest import golden_index
    meta = golden_index()[name]
    d, data, cfg = _setup(tmp_path, name, meta['block_shape'])
    c = MergeAssignmentsLocal.default_task_config()
    c['reference_empty_job_quirk'] = True
    _write_task_config(cfg, 'merge_assignments', c)
    if gpus > 1:
        # the z-slab path cannot emulate the quirk; the job must not silently drop it
        from cluster_tools_amd.thresholded_components.block_components import BlockComponentsLocal
        bc = BlockComponentsLocal.default_task_config()
        bc.update({'gpus': gpus, 'dist_backend': 'gloo'})
        _write_task_config(cfg, 'block_components', bc)
    t = ThresholdedComponentsWorkflow(tmp_folder=str(tmp_path / 'tmp'), config_dir=cfg, target='local',
                                      max_jobs=meta['n_jobs_block_faces'], input_path=data,
                                      input_key='volumes/boundaries', output_path=data, output_key='data',
                                      assignment_key='assignments', threshold=float(d['threshold']),
                                      threshold_mode=meta['mode'])
    assert _build([t], tmp_path / 'tmp')
    with n5.open_file(data, 'r') as f:
        np.testing.assert_array_equal(O.canon(f['data'][:]), d['labels_canon'])
        np.testing.assert_array_equal(O.canon(f['assignments'][:]), d['lut_canon'])


@pytest.mark.parametrize('name', ['bmap_less', 'bmap_mask', 'bmap_greater'])
def test_workflow_sharded_two_ranks(tmp_path, name):
    """block_components config gpus = 2: the fused job starts two z-slab ranks
    (torch.distributed.run, gloo collectives staged through the host: both ranks share this one
    GPU, which RCCL refuses) and assembles the reference's artefacts from them."""
    from cluster_tools_amd import n5
    from cluster_tools_amd.thresholded_components import ThresholdedComponentsWorkflow
    from cluster_tools_amd.thresholded_components.block_components import BlockComponentsLocal
    from conftest import golden_index
    meta = golden_index()[name]
    d, data, cfg = _setup(tmp_path, name, meta['block_shape'])
    c = BlockComponentsLocal.default_task_config()
    c.update({'gpus': 2, 'dist_backend': 'gloo'})
    _write_task_config(cfg, 'block_components', c)
    kw = dict(mask_path=data, mask_key='volumes/mask') if 'mask' in d else {}
    t = ThresholdedComponentsWorkflow(tmp_folder=str(tmp_path / 'tmp'), config_dir=cfg, target='local', max_jobs=4,
                                      input_path=data, input_key='volumes/boundaries', output_path=data,
                                      output_key='data', assignment_key='assignments',
                                      threshold=float(d['threshold']), threshold_mode=meta['mode'], **kw)
    assert _build([t], tmp_path / 'tmp')
    with n5.open_file(data, 'r') as f:
        seg = f['data'][:]
        np.testing.assert_array_equal(O.canon(seg), d['labels_canon'])
        np.testing.assert_array_equal(O.canon(f['assignments'][:]), d['lut_canon'])
        assert f['data'].attrs['maxId'] == int(d['max_id'])
    ref = O.label_volume(d['input'], meta['block_shape'], float(d['threshold']), meta['mode'], d.get('mask'))
    np.testing.assert_array_equal(seg, ref['labels'])          # raw ids too (min-id representatives)
    off = json.load(open(str(tmp_path / 'tmp' / 'cc_offsets.json')))
    np.testing.assert_array_equal(np.array(off['offsets'], dtype=np.uint64), d['offsets'])
    timing = json.load(open(str(tmp_path / 'tmp' / 'cc_fused_timing.json')))
    assert timing['gpus'] == 2


@pytest.mark.slow
@pytest.mark.parametrize('mode', ['greater', 'less'])
def test_workflow_c1(tmp_path, mode):
    """BASELINE config 1 through the drop-in API: a CREMI-sized (125, 1250, 1250) float32 N5
    dataset (synthetic: the CREMI sample is absent), block_shape [50, 512, 512] (the reference
    default), threshold 0.5, target 'local'; the N5 output against the oracle, and the host /
    device split recorded by the fused job."""
    import torch
    from cluster_tools_amd import n5, _lib
    from cluster_tools_amd.cluster_tasks import BaseClusterTask
    from cluster_tools_amd.thresholded_components import ThresholdedComponentsWorkflow
    shape, bs = (125, 1250, 1250), [50, 512, 512]
    with _lib.Context(0) as ctx:
        x = ctx.generate_boundary_map(shape).cpu().numpy()
    data = str(tmp_path / 'c1.n5')
    with n5.open_file(data) as f:
        f.create_dataset('volumes/raw/boundaries', data=x, chunks=(25, 256, 256), compression='gzip')
    cfg = str(tmp_path / 'config')
    os.makedirs(cfg)
    g = BaseClusterTask.default_global_config()
    assert g['block_shape'] == bs
    with open(os.path.join(cfg, 'global.config'), 'w') as f:
        json.dump(g, f)
    t = ThresholdedComponentsWorkflow(tmp_folder=str(tmp_path / 'tmp'), config_dir=cfg, target='local', max_jobs=16,
                                      input_path=data, input_key='volumes/raw/boundaries', output_path=data,
                                      output_key='segmentation/cc', assignment_key='segmentation/assignments',
                                      threshold=0.5, threshold_mode=mode)
    assert _build([t], tmp_path / 'tmp')
    ref = O.label_volume(x, bs, 0.5, mode, n_threads=16)
    with n5.open_file(data, 'r') as f:
        seg = f['segmentation/cc'][:]
        assert f['segmentation/cc'].chunks == (25, 256, 256)
        assert f['segmentation/cc'].attrs['maxId'] == ref['max_id']
        np.testing.assert_array_equal(f['segmentation/assignments'][:], ref['lut'])
    np.testing.assert_array_equal(seg, ref['labels'])
    timing = json.load(open(str(tmp_path / 'tmp' / 'cc_fused_timing.json')))
    for k in ('n5_read_s', 'h2d_device_d2h_s', 'n5_write_s'):
        assert timing[k] > 0
    # the one-shot jobs run without torch (cc_label_volume_host on numpy buffers, host-only
    # cc_merge_offsets); the other stages skip the device after the fused job
    assert timing['torch_imported'] is False
    print('C1 %s timing: %s' % (mode, timing))


def test_integration_binding_runs_as_documented():
    """INTEGRATION.md section B executed as written (the ctypes binding a maintainer would add to
    the reference): label_volume on a golden volume against the oracle and the reference's
    artefacts, then the Threshold and evaluation snippets in the same namespace."""
    import ctypes
    import torch
    from conftest import exec_integration_binding, integration_blocks, golden_index
    ns = exec_integration_binding()
    name = 'bmap_mask'
    meta, d = golden_index()[name], load_golden(name)
    out, values, lut, max_id = ns['label_volume'](d['input'], meta['block_shape'], float(d['threshold']),
                                                   meta['mode'], mask=d['mask'])
    r = O.label_volume(d['input'], meta['block_shape'], float(d['threshold']), meta['mode'], d['mask'])
    np.testing.assert_array_equal(out, r['labels'])
    np.testing.assert_array_equal(values, d['block_values'])
    np.testing.assert_array_equal(lut, r['lut'])
    assert max_id == int(d['max_id'])
    # the Threshold / evaluation blocks extend the same module namespace
    for b in integration_blocks():
        if 'def threshold_volume' in b or 'def measures_on_device' in b or 'def watershed_from_seeds' in b:
            exec(compile(b, 'INTEGRATION.md', 'exec'), ns)
    L = ns['_L']
    ctx = ctypes.c_void_p()
    assert L.cc_create(0, ctypes.byref(ctx)) == 0
    try:
        x = torch.from_numpy(d['input']).cuda()
        got = torch.empty(x.shape, dtype=torch.uint8, device='cuda')
        torch.cuda.synchronize()
        ns['threshold_volume'](ctx, x.data_ptr(), x.shape, meta['block_shape'], float(d['threshold']),
                               meta['mode'], got.data_ptr())
        want = O.threshold_volume(d['input'], meta['block_shape'], float(d['threshold']), meta['mode'])
        np.testing.assert_array_equal(got.cpu().numpy(), want)
        seg = torch.from_numpy(out.view(np.int64)).cuda()
        torch.cuda.synchronize()
        m = ns['measures_on_device'](ctx, seg.data_ptr(), seg.data_ptr(), seg.shape, meta['block_shape'])
        assert abs(m['rand-index'] - 1.0) < 1e-12 and abs(m['vi-split']) < 1e-12 and abs(m['vi-merge']) < 1e-12
        # the watershed block: the labels as seeds, grown over the input (oracle/watershed.py)
        from oracle import watershed as W
        ws = torch.empty_like(seg)
        mk = torch.from_numpy((d['mask'] != 0).astype(np.uint8)).cuda()
        torch.cuda.synchronize()
        ns['watershed_from_seeds'](ctx, x.data_ptr(), seg.data_ptr(), mk.data_ptr(), x.shape, meta['block_shape'],
                                   ws.data_ptr())
        want = W.watershed_from_seeds(d['input'], out, meta['block_shape'], (d['mask'] != 0).astype(np.uint8))
        np.testing.assert_array_equal(ws.cpu().numpy().view(np.uint64), want)
        # the 4-D block (cc_normalize_channels + CC_OPT_WS_PRENORMALIZED): two channels, max
        for b in integration_blocks():
            if 'def watershed_4d' in b:
                exec(compile(b, 'INTEGRATION.md', 'exec'), ns)
        x4 = np.stack([d['input'], d['input'][:, ::-1, :].copy()])
        s4 = torch.from_numpy(x4).cuda()
        tmp = torch.empty(x.shape, dtype=torch.float32, device='cuda')
        torch.cuda.synchronize()
        ns['watershed_4d'](ctx, s4.data_ptr(), 2, x.shape, meta['block_shape'], 'max', tmp.data_ptr(), seg.data_ptr(),
                           mk.data_ptr(), ws.data_ptr())
        want = W.watershed_from_seeds(x4, out, meta['block_shape'], (d['mask'] != 0).astype(np.uint8), 0, None, 'max')
        np.testing.assert_array_equal(ws.cpu().numpy().view(np.uint64), want)
    finally:
        L.cc_destroy(ctx)


@pytest.mark.parametrize('gpus', [1, 2])
def test_workflow_resized_mask(tmp_path, gpus):
    """A mask dataset at half resolution (block_components.py:274-275 -> ResizedVolume order 0):
    the workflow output equals the oracle labelling with the mask resized by the documented
    nearest-neighbour rule (parity with elf unpinned), on one GPU and over two z-slab ranks."""
    from cluster_tools_amd import n5
    from cluster_tools_amd.thresholded_components import ThresholdedComponentsWorkflow
    from cluster_tools_amd.thresholded_components.block_components import BlockComponentsLocal
    name, bs = 'bmap_greater', (16, 32, 32)
    d, data, cfg = _setup(tmp_path, name, bs)
    shape = d['input'].shape
    low = (np.random.default_rng(4).random(tuple(-(-s // 2) for s in shape)) < 0.7).astype(np.uint8)
    with n5.open_file(data) as f:
        f.create_dataset('volumes/mask_s1', data=low, chunks=(8, 16, 16), compression='gzip')
    if gpus > 1:
        c = BlockComponentsLocal.default_task_config()
        c.update({'gpus': gpus, 'dist_backend': 'gloo'})
        _write_task_config(cfg, 'block_components', c)
    t = ThresholdedComponentsWorkflow(tmp_folder=str(tmp_path / 'tmp'), config_dir=cfg, target='local', max_jobs=4,
                                      input_path=data, input_key='volumes/boundaries', output_path=data,
                                      output_key='data', assignment_key='assignments', threshold=0.5,
                                      threshold_mode='greater', mask_path=data, mask_key='volumes/mask_s1')
    assert _build([t], tmp_path / 'tmp')
    ref = O.label_volume(d['input'], bs, 0.5, 'greater', O.resize_mask_nearest(low, shape))
    with n5.open_file(data, 'r') as f:
        np.testing.assert_array_equal(f['data'][:], ref['labels'])
        np.testing.assert_array_equal(f['assignments'][:], ref['lut'])


@pytest.mark.parametrize('name', ['bmap_less', 'bmap_mask_less', 'inf_block'])
def test_threshold_and_watershed_workflow(tmp_path, name):
    """ThresholdAndWatershedWorkflow (thresholded_components_workflow.py:107-144): the components,
    then WatershedFromSeeds grows them over the input in place.  Against the oracle chain (the C
    oracle's labels as seeds -> oracle/watershed.py); the watershed itself is parity unpinned
    (the reference's vu.watershed does not exist)."""
    from cluster_tools_amd import n5
    from cluster_tools_amd.thresholded_components.thresholded_components_workflow import \
        ThresholdAndWatershedWorkflow
    from conftest import golden_index
    from oracle import watershed as W
    meta = golden_index()[name]
    bs = meta['block_shape']
    d, data, cfg = _setup(tmp_path, name, bs)
    kw = {}
    mask = d.get('mask')
    if mask is not None:
        kw = dict(mask_path=data, mask_key='volumes/mask')
    t = ThresholdAndWatershedWorkflow(tmp_folder=str(tmp_path / 'tmp'), config_dir=cfg, target='local', max_jobs=4,
                                      input_path=data, input_key='volumes/boundaries', output_path=data,
                                      output_key='data', assignment_key='assignments',
                                      threshold=float(d['threshold']), threshold_mode=meta['mode'], **kw)
    assert _build([t], tmp_path / 'tmp')
    with n5.open_file(data, 'r') as f:
        ws = f['data'][:]
    seeds = O.label_volume(d['input'], bs, float(d['threshold']), meta['mode'], mask, n_threads=4)['labels']
    want = W.watershed_from_seeds(d['input'], seeds, bs, None if mask is None else (mask != 0).astype(np.uint8))
    if mask is not None:          # blocks without a mask voxel are skipped: they keep the seeds (0 there)
        m = (mask != 0)
        Z, Y, X = ws.shape
        for z0 in range(0, Z, bs[0]):
            for y0 in range(0, Y, bs[1]):
                for x0 in range(0, X, bs[2]):
                    bb = np.s_[z0:z0 + bs[0], y0:y0 + bs[1], x0:x0 + bs[2]]
                    if not m[bb].any():
                        want[bb] = seeds[bb]
    np.testing.assert_array_equal(ws, want)
    assert (tmp_path / 'tmp' / 'watershed_from_seeds.log').exists()


@pytest.mark.parametrize('agg', ['mean', 'max'])
def test_threshold_and_watershed_workflow_channels(tmp_path, agg):
    """ThresholdAndWatershedWorkflow with `channel` on a 4-D (C, Z, Y, X) input: the components
    from that channel (block_components.py:150-159), the watershed over _read_data's values
    (the channels channel_begin:channel_end of each block normalized together, then
    agglomerate_channels: watershed_from_seeds.py:127-139) -- against the oracle chain."""
    import json
    import os
    from cluster_tools_amd import n5
    from cluster_tools_amd.thresholded_components.thresholded_components_workflow import \
        ThresholdAndWatershedWorkflow
    from oracle import watershed as W
    shape, bs = (32, 64, 80), [16, 32, 40]
    x4 = np.stack([O.boundary_map(shape, origin=(0, 5 * c, 9 * c)) for c in range(3)])
    data = str(tmp_path / 'data.n5')
    with n5.open_file(data, 'a') as f:
        f.create_dataset('volumes/boundaries', data=x4, chunks=(1, 16, 32, 40), compression='gzip')
    from cluster_tools_amd.cluster_tasks import BaseClusterTask
    cfg = str(tmp_path / 'config')
    os.makedirs(cfg, exist_ok=True)
    g = BaseClusterTask.default_global_config()
    g['block_shape'] = bs
    with open(os.path.join(cfg, 'global.config'), 'w') as fh:
        json.dump(g, fh)
    with open(os.path.join(cfg, 'watershed_from_seeds.config'), 'w') as fh:
        json.dump({'channel_begin': 0, 'channel_end': 2, 'agglomerate_channels': agg}, fh)
    t = ThresholdAndWatershedWorkflow(tmp_folder=str(tmp_path / 'tmp'), config_dir=cfg, target='local', max_jobs=4,
                                      input_path=data, input_key='volumes/boundaries', output_path=data,
                                      output_key='data', assignment_key='assignments', threshold=0.5,
                                      threshold_mode='less', channel=1)     # luigi.IntParameter upstream
    assert _build([t], tmp_path / 'tmp')
    with n5.open_file(data, 'r') as f:
        ws = f['data'][:]
    seeds = O.label_volume(np.ascontiguousarray(x4[1]), bs, 0.5, 'less', n_threads=4)['labels']
    want = W.watershed_from_seeds(x4, seeds, bs, None, 0, 2, agg)
    np.testing.assert_array_equal(ws, want)


def test_watershed_job_block_subset(tmp_path):
    """The WatershedFromSeeds job over a subset of the blocks reads and grows only their bounding
    box: the listed blocks equal the oracle's, the others stay as they were (zeros)."""
    import json
    from cluster_tools_amd import n5
    from cluster_tools_amd.watershed.watershed_from_seeds import watershed_from_seeds
    from oracle import watershed as W
    shape, bs = (40, 72, 88), [16, 32, 40]
    x = O.boundary_map(shape, origin=(1, 2, 3))
    seeds = O.label_volume(x, bs, 0.5, 'less', n_threads=4)['labels']
    data = str(tmp_path / 'data.n5')
    with n5.open_file(data, 'a') as f:
        f.create_dataset('x', data=x, chunks=(8, 16, 20), compression='gzip')
        f.create_dataset('seeds', data=seeds, chunks=(8, 16, 20), compression='gzip')
        f.create_dataset('ws', shape=shape, chunks=(8, 16, 20), compression='gzip', dtype='uint64')
    blocks = [4, 5, 13]                               # 3 x 3 x 3 blocks
    cfg = str(tmp_path / 'watershed_from_seeds_job_0.config')
    with open(cfg, 'w') as fh:
        json.dump({'input_path': data, 'input_key': 'x', 'seeds_path': data, 'seeds_key': 'seeds',
                   'output_path': data, 'output_key': 'ws', 'block_shape': bs, 'block_list': blocks}, fh)
    watershed_from_seeds(0, cfg)
    with n5.open_file(data, 'r') as f:
        ws = f['ws'][:]
    want = W.watershed_from_seeds(x, seeds, bs)
    from cluster_tools_amd.utils import volume_utils as vu
    blocking = vu.Blocking([0, 0, 0], shape, bs)
    covered = np.zeros(shape, dtype=bool)
    for b in blocks:
        bb = vu.block_to_bb(blocking.getBlock(b))
        np.testing.assert_array_equal(ws[bb], want[bb])
        covered[bb] = True
    assert not ws[~covered].any()
