#! /usr/bin/python
"""BlockComponents task + job (reference: cluster_tools/thresholded_components/block_components.py).

Task parameters, configs, output dataset (uint64, chunks block//2, gzip), the per-job offsets
JSON and the log contract are the reference's (block_components.py:21-119,236-291).  The job's
compute runs on the MI355X through libcc_mi355x (4-D input with `channel`: cc_channel_mean first;
sigma_prefilter > 0: cc_gaussian_smooth_blocks first):
  fused=False  cc_block_components: block-local 26-connected labels in skimage numbering and
               the per-block values (n_i + 1 or 0), exactly what the reference job writes;
  fused=True   (set by ThresholdedComponentsWorkflow) cc_label_volume: all five stages in this
               job; the output dataset receives the FINAL labels and the downstream tasks only
               emit their artefacts (cc_offsets.json, the assignments LUT, maxId, logs).
               Task config 'gpus' > 1 shards the volume in z-slabs over that many GPUs
               (sharded_job.py, one rank per GPU, RCCL).
One job labels the whole volume; per-block results do not depend on the job split.  N5 chunks
are coded natively (cc_n5_read / cc_n5_write on host threads); the fused job records its
n5-read / H2D / device / D2H / n5-write split in <tmp>/cc_fused_timing.json.
"""
import json
import os
import sys
import time

import numpy as np

from cluster_tools_amd.luigi_compat import Task, Parameter, FloatParameter, TaskParameter, BoolParameter
from cluster_tools_amd.cluster_tasks import LocalTask
import cluster_tools_amd.utils.volume_utils as vu
import cluster_tools_amd.utils.function_utils as fu

FUSED_MARKER = 'cc_fused.json'
FUSED_LUT = 'cc_fused_assignments.npy'
FUSED_TIMING = 'cc_fused_timing.json'     # host / device split of the fused job (seconds)


class BlockComponentsBase(Task):
    task_name = 'block_components'
    src_file = os.path.abspath(__file__)
    allow_retry = False

    input_path = Parameter()
    input_key = Parameter()
    output_path = Parameter()
    output_key = Parameter()
    dependency = TaskParameter()
    threshold = FloatParameter()
    threshold_mode = Parameter(default='greater')
    mask_path = Parameter(default='')
    mask_key = Parameter(default='')
    channel = Parameter(default=None)
    fused = BoolParameter(default=False)

    threshold_modes = ('greater', 'less', 'equal')

    @staticmethod
    def default_task_config():
        # gpus: GPUs of this node for the fused job (> 1: z-slab sharding, one rank per GPU);
        # dist_backend: 'nccl' (RCCL over xGMI) or 'gloo' (host-staged, rehearsal on one GPU)
        config = LocalTask.default_task_config()
        config.update({'sigma_prefilter': 0, 'gpus': 1, 'dist_backend': 'nccl'})
        return config

    def requires(self):
        return self.dependency

    def run_impl(self):
        shebang, block_shape, roi_begin, roi_end = self.global_config_values()
        self.init(shebang)
        shape = vu.get_shape(self.input_path, self.input_key)
        assert self.threshold_mode in self.threshold_modes
        config = self.get_task_config()
        config.update({'input_path': self.input_path, 'input_key': self.input_key,
                       'output_path': self.output_path, 'output_key': self.output_key,
                       'block_shape': block_shape, 'tmp_folder': self.tmp_folder,
                       'threshold': self.threshold, 'threshold_mode': self.threshold_mode,
                       'fused': bool(self.fused)})
        if self.mask_path != '':
            assert self.mask_key != ''
            config.update({'mask_path': self.mask_path, 'mask_key': self.mask_key})
        chunks = config.pop('chunks', None)
        if chunks is None:
            chunks = tuple(bs // 2 for bs in block_shape)
        if self.channel is None:
            assert len(shape) == 3, str(len(shape))
        else:
            # 4-D (C, Z, Y, X) input: the listed channels are averaged (block_components.py:75-89)
            assert len(shape) == 4, str(len(shape))
            chans = channel_list(self.channel)
            assert all(0 <= c < shape[0] for c in chans), (shape[0], chans)
            shape = shape[1:]
            config.update({'channel': self.channel})
        chunks = tuple(max(1, min(ch, sh)) for ch, sh in zip(chunks, shape))
        compression = config.pop('compression', 'gzip')
        # the reference empty-job branch (merge_assignments config, see merge_assignments.py) is
        # applied here when the whole path runs fused in this job
        from cluster_tools_amd.thresholded_components.merge_assignments import QUIRK_KEY
        ma_cfg = os.path.join(self.config_dir, 'merge_assignments.config')
        if self.fused and os.path.exists(ma_cfg):
            with open(ma_cfg) as f:
                if json.load(f).get(QUIRK_KEY, False):
                    config['quirk_jobs'] = int(self.max_jobs)
        with vu.file_reader(self.output_path) as f:
            f.require_dataset(self.output_key, shape=shape, dtype='uint64', compression=compression, chunks=chunks)
        block_list = vu.blocks_in_volume(shape, block_shape, roi_begin, roi_end)
        n_jobs = 1
        self.prepare_jobs(n_jobs, block_list, config)
        self.submit_jobs(n_jobs)
        self.wait_for_jobs()
        self.check_jobs(n_jobs)


class BlockComponentsLocal(BlockComponentsBase, LocalTask):
    pass


def _n_threads():
    return max(1, min(16, len(os.sched_getaffinity(0))))


def _read(path, key, box=None, dtype=None):
    """Region of an N5 dataset through the native codec (whole dataset when box is None)."""
    with vu.file_reader(path, 'r') as f:
        ds = f[key]
        ds.n_threads = _n_threads()
        a = ds.read_region(box or [(0, s) for s in ds.shape])
    return a if dtype is None else a.astype(dtype, copy=False)


def read_mask(config, shape, box=None):
    """The job's mask on the host: (uint8 array, resized).  A full-resolution mask is read over
    `box`; a mask of another shape (vu.ResizedMask) is read whole and resized on the device by
    device_mask (cc_resize_mask_nearest).  (None, False) without a mask."""
    if not config.get('mask_path', ''):
        return None, False
    m = vu.load_mask(config['mask_path'], config['mask_key'], shape)
    resized = isinstance(m, vu.ResizedMask)
    a = _read(config['mask_path'], config['mask_key'], None if resized else box)
    return (a != 0).astype(np.uint8), resized


def device_mask(ctx, mask, resized, shape, dev, z0=0, nz=None):
    """uint8 CUDA mask of the (slab of the) volume from read_mask's result."""
    import torch
    if mask is None:
        return None
    if resized:
        return ctx.resize_mask(mask, shape, z0, nz)
    return torch.from_numpy(mask).to(dev)


def channel_list(channel):
    """The reference's `channel` (int or list of ints, block_components.py:152) as a list; a
    JSON / luigi round trip may hand it over as a string."""
    if isinstance(channel, str):
        channel = json.loads(channel)
    if isinstance(channel, (int, np.integer)):
        return [int(channel)]
    return [int(c) for c in channel]


def read_input(config, box=None):
    """Host side of the job input: the float32 volume (3-D input; normalize's astype('float32'),
    volume_utils.py:99, done on the host), or for 4-D input with config['channel'] the distinct
    listed channels of the region in the dataset's dtype plus the list as indices into that stack
    (averaged on the device by to_device)."""
    channel = config.get('channel')
    if channel is None:
        return _read(config['input_path'], config['input_key'], box, dtype=np.float32), None
    chans = channel_list(channel)
    distinct = sorted(set(chans))
    with vu.file_reader(config['input_path'], 'r') as f:
        ds = f[config['input_key']]
        ds.n_threads = _n_threads()
        box = box or [(0, s) for s in ds.shape[1:]]
        stack = np.empty((len(distinct),) + tuple(e - b for b, e in box), dtype=ds.dtype)
        for i, c in enumerate(distinct):
            stack[i] = ds.read_region([(c, c + 1)] + list(box))[0]
    return stack, [distinct.index(c) for c in chans]


def to_device(ctx, host, chans, dev, config=None):
    """float32 device volume for the labelling: upload, and for a channel stack the mean of the
    listed channels (cc_channel_mean: np.mean(axis=0) as block_components.py:150-159 does it);
    then the sigma_prefilter front (prefilter)."""
    import torch
    x = torch.from_numpy(host).to(dev) if chans is None else ctx.channel_mean(host, chans)
    return prefilter(ctx, x, config)


def prefilter(ctx, x, config):
    """config['sigma_prefilter'] > 0: per block normalize -> Gaussian smoothing in place
    (block_components.py:160-163; cc_gaussian_smooth_blocks, the filter restating vigra's).  The
    second normalize is the labelling's own."""
    sigma = float((config or {}).get('sigma_prefilter', 0) or 0)
    if sigma > 0:
        x = ctx.gaussian_smooth_blocks(x, config['block_shape'], sigma, out=x)
    return x


def _write_output(config, labels, box, n_threads=None):
    """Final / block-local labels into the output dataset.  Chunks of empty blocks are not
    created (the reference skips empty blocks, block_components.py:175-177, and they read as 0)."""
    with vu.file_reader(config['output_path']) as f:
        ds = f[config['output_key']]
        ds.n_threads = n_threads or _n_threads()
        ds.write_region(box, labels, skip_zero_chunks=True)


def _write_fused_artefacts(tmp_folder, config, values, lut, res, timing):
    np.save(os.path.join(tmp_folder, FUSED_LUT), lut)
    with open(os.path.join(tmp_folder, FUSED_MARKER), 'w') as f:
        json.dump({'output_path': os.path.abspath(config['output_path']),
                   'output_key': config['output_key'], 'n_labels': int(res['n_labels']),
                   'max_id': int(res['max_id']), 'n_components': int(res['n_components'])}, f)
    with open(os.path.join(tmp_folder, FUSED_TIMING), 'w') as f:
        json.dump(timing, f, indent=1)
    fu.log('timing (s): ' + ', '.join('%s %.3f' % (k, v) for k, v in timing.items() if k.endswith('_s')))


def _fused_host(config, shape, nb, inp, mask, timing):
    """The common case of the fused job -- 3-D float input, no resized mask, no prefilter -- with
    no torch in the process: numpy buffers straight through cc_label_volume_host (H2D, the five
    stages, D2H in one call on the system HIP runtime).  The torch import is most of a one-shot
    job's wall time."""
    from cluster_tools_amd import _lib
    _lib.load(host_only=True)
    device = int(os.environ.get('CC_DEVICE', '0'))
    t = time.perf_counter()
    with _lib.Context(device) as ctx:
        timing['ctx_init_s'] = time.perf_counter() - t
        ctx.set_empty_job_quirk(config.get('quirk_jobs', 0))
        t = time.perf_counter()
        labels, res = ctx.label_volume(inp, config['block_shape'], config['threshold'], config['threshold_mode'],
                                       mask=mask)
        timing['h2d_device_d2h_s'] = time.perf_counter() - t
        values = ctx.block_values(nb)
        lut = ctx.lut(res['n_labels'])
    del inp, mask
    t = time.perf_counter()
    _write_output(config, labels, [(0, s) for s in shape])
    timing['n5_write_s'] = time.perf_counter() - t
    timing['torch_imported'] = 'torch' in sys.modules
    if res.get('identity_lut'):
        fu.log('a block_faces job has no pairs: no merge (reference empty-job branch)')
    return values, lut, res, timing


def _fused_single(config, shape, nb):
    """All five stages on one GPU, with the host side split out: N5 read, H2D, device, D2H, N5
    write (the PCIe-inclusive and codec-inclusive rates are reported beside the
    device-resident one)."""
    timing = {'voxels': int(np.prod(shape)), 'gpus': 1}
    t = time.perf_counter()
    inp, chans = read_input(config)
    mask, resized = read_mask(config, shape)
    timing['n5_read_s'] = time.perf_counter() - t
    sigma = float(config.get('sigma_prefilter', 0) or 0)
    if chans is None and not resized and sigma <= 0 and not config.get('torch_path', False):
        return _fused_host(config, shape, nb, inp, mask, timing)
    import torch
    from cluster_tools_amd import _lib
    device = int(os.environ.get('CC_DEVICE', '0'))
    dev = torch.device('cuda', device)
    torch.cuda.set_device(dev)
    with _lib.Context(device) as ctx:
        ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        ctx.set_empty_job_quirk(config.get('quirk_jobs', 0))
        t = time.perf_counter()
        if chans is None:
            x = torch.from_numpy(inp).to(dev)
        else:
            x = torch.from_numpy(inp.reshape(-1).view(np.uint8)).to(dev)
        m = device_mask(ctx, mask, resized, shape, dev)
        torch.cuda.synchronize(dev)
        timing['h2d_s'] = time.perf_counter() - t
        stack_shape, stack_dtype = inp.shape, inp.dtype
        del inp, mask
        t = time.perf_counter()
        if chans is not None:
            x = ctx.channel_mean(x, chans, shape4=stack_shape, dtype=stack_dtype)
        x = prefilter(ctx, x, config)
        labels_dev, res = ctx.label_volume(x, config['block_shape'], config['threshold'],
                                           config['threshold_mode'], m)
        torch.cuda.synchronize(dev)
        timing['device_s'] = time.perf_counter() - t
        values = ctx.block_values(nb)
        lut = ctx.lut(res['n_labels'])
    del x, m
    t = time.perf_counter()
    labels = labels_dev.cpu().numpy().view(np.uint64)
    timing['d2h_s'] = time.perf_counter() - t
    del labels_dev
    t = time.perf_counter()
    _write_output(config, labels, [(0, s) for s in shape])
    timing['n5_write_s'] = time.perf_counter() - t
    if res.get('identity_lut'):
        fu.log('a block_faces job has no pairs: no merge (reference empty-job branch)')
    return values, lut, res, timing


def _free_port():
    import socket
    with socket.socket() as sk:
        sk.bind(('127.0.0.1', 0))
        return sk.getsockname()[1]


def _fused_sharded(config_path, config, shape, nb):
    """config['gpus'] > 1: z-slab sharding over that many GPUs of this node.  This
    job process has not touched a GPU; it starts one rank per GPU with torch.distributed.run
    (cluster_tools_amd/thresholded_components/sharded_job.py; RCCL collectives, or gloo with
    config['dist_backend'] = 'gloo' to rehearse on one device) and assembles the per-rank block
    values and LUT parts into the reference's artefacts.  This replaces the reference's
    ProcessPool of block jobs (cluster_tasks.py:301-335, 545-551) with one rank per GPU."""
    import subprocess
    from cluster_tools_amd.distributed import assemble_lut
    bz = config['block_shape'][0]
    world = max(1, min(int(config['gpus']), -(-shape[0] // bz)))
    out_dir = os.path.join(config['tmp_folder'], 'cc_shards')
    os.makedirs(out_dir, exist_ok=True)
    for fn in os.listdir(out_dir):
        os.remove(os.path.join(out_dir, fn))
    import cluster_tools_amd
    pkg = os.path.dirname(os.path.abspath(cluster_tools_amd.__file__))
    # (this module runs as a copy in the tmp folder: locate the package, not __file__)
    script = os.path.join(pkg, 'thresholded_components', 'sharded_job.py')
    repo = os.path.dirname(pkg)
    env = dict(os.environ)
    env['PYTHONPATH'] = repo + (os.pathsep + env['PYTHONPATH'] if env.get('PYTHONPATH') else '')
    env['HSA_ENABLE_IPC_MODE_LEGACY'] = '0'
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', str(world),
           '--master-addr', '127.0.0.1', '--master-port', str(_free_port()), script, config_path, out_dir]
    fu.log('z-slab sharded run on %i GPUs (%s)' % (world, config.get('dist_backend', 'nccl')))
    t = time.perf_counter()
    subprocess.run(cmd, check=True, env=env)
    wall = time.perf_counter() - t
    parts = [np.load(os.path.join(out_dir, 'rank_%i.npz' % r)) for r in range(world)]
    sums = [int(p['sum']) for p in parts]
    values = np.concatenate([p['values'] for p in parts])
    assert len(values) == nb, (len(values), nb)
    lut = assemble_lut([p['lut'] for p in parts], sums)
    n_labels = sum(sums) + 1
    res = {'n_labels': n_labels, 'max_id': n_labels - 1,
           'n_components': int(sum(int(p['n_components']) for p in parts))}
    timing = {'voxels': int(np.prod(shape)), 'gpus': world, 'ranks_wall_s': wall}
    for k in parts[0].files:
        if k.endswith('_s'):
            timing[k] = max(float(p[k]) for p in parts)          # slowest rank per stage
    return values, lut, res, timing


def block_components(job_id, config_path):
    fu.log('start processing job %i' % job_id)
    fu.log('reading config from %s' % config_path)
    with open(config_path) as f:
        config = json.load(f)
    block_list = config['block_list']
    tmp_folder = config['tmp_folder']
    block_shape = config['block_shape']
    threshold, mode = config['threshold'], config['threshold_mode']
    fused = config.get('fused', False)
    fu.log('Applying threshold %f with mode %s' % (threshold, mode))
    shape = tuple(vu.get_shape(config['input_path'], config['input_key']))
    if config.get('channel') is not None:
        shape = shape[1:]
    nb = vu.Blocking([0, 0, 0], list(shape), block_shape).numberOfBlocks

    if fused:
        sharded = int(config.get('gpus', 1)) > 1
        if sharded and int(config.get('quirk_jobs', 0)) > 0:
            # the empty-job emulation (merge_assignments.py:115-123) needs every block's face-pair
            # flag in one place: it runs on the single-volume fused path only
            fu.log('reference_empty_job_quirk is set: running on one GPU instead of %i z-slab ranks'
                   % int(config['gpus']))
            sharded = False
        if sharded:
            values, lut, res, timing = _fused_sharded(config_path, config, shape, nb)
        else:
            values, lut, res, timing = _fused_single(config, shape, nb)
        _write_fused_artefacts(tmp_folder, config, values, lut, res, timing)
    else:
        import torch
        from cluster_tools_amd import _lib
        inp, chans = read_input(config)
        mask, resized = read_mask(config, shape)
        with _lib.Context(int(os.environ.get('CC_DEVICE', '0'))) as ctx:
            x = to_device(ctx, inp, chans, ctx.torch_device(), config)
            m = device_mask(ctx, mask, resized, shape, x.device)
            lab_dev, values = ctx.block_components(x, block_shape, threshold, mode, m)
            labels = lab_dev.cpu().numpy().view(np.uint64)
        _write_output(config, labels, [(0, s) for s in shape])
    for b in block_list:
        fu.log_block_success(b)
    offsets = {b: int(values[b]) for b in block_list}
    with open(os.path.join(tmp_folder, 'connected_components_offsets_%i.json' % job_id), 'w') as f:
        json.dump(offsets, f)
    fu.log_job_success(job_id)


if __name__ == '__main__':
    path = sys.argv[1]
    assert os.path.exists(path), path
    job_id = int(os.path.split(path)[1].split('.')[0].split('_')[-1])
    block_components(job_id, path)
