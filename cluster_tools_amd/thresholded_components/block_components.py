#! /usr/bin/python
"""BlockComponents task + job (reference: cluster_tools/thresholded_components/block_components.py).

Task parameters, configs, output dataset (uint64, chunks block//2, gzip), the per-job offsets
JSON and the log contract are the reference's (block_components.py:21-119,236-291).  The job's
compute runs on the MI355X through libcc_mi355x:
  fused=False  cc_block_components: block-local 26-connected labels in skimage numbering and
               the per-block values (n_i + 1 or 0), exactly what the reference job writes;
  fused=True   (set by ThresholdedComponentsWorkflow) cc_label_volume: all five stages in this
               job; the output dataset receives the FINAL labels and the downstream tasks only
               emit their artefacts (cc_offsets.json, the assignments LUT, maxId, logs).
One GPU job labels the whole volume; per-block results do not depend on the job split.
"""
import json
import os
import sys

import numpy as np

from cluster_tools_amd.luigi_compat import Task, Parameter, FloatParameter, TaskParameter, BoolParameter
from cluster_tools_amd.cluster_tasks import LocalTask
import cluster_tools_amd.utils.volume_utils as vu
import cluster_tools_amd.utils.function_utils as fu

FUSED_MARKER = 'cc_fused.json'
FUSED_LUT = 'cc_fused_assignments.npy'


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
        config = LocalTask.default_task_config()
        config.update({'sigma_prefilter': 0})
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
        if self.channel is not None:
            raise NotImplementedError('channel != None (4-D input) is not supported on the MI355X path')
        assert len(shape) == 3, str(len(shape))
        if config.get('sigma_prefilter', 0) > 0:
            raise NotImplementedError('sigma_prefilter > 0 is not supported on the MI355X path')
        chunks = tuple(max(1, min(ch, sh)) for ch, sh in zip(chunks, shape))
        compression = config.pop('compression', 'gzip')
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


def _load(path, key, dtype=None):
    with vu.file_reader(path, 'r') as f:
        a = f[key][:]
    return a if dtype is None else a.astype(dtype, copy=False)


def block_components(job_id, config_path):
    import torch
    from cluster_tools_amd import _lib
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

    inp = _load(config['input_path'], config['input_key'], np.float32)
    shape = inp.shape
    mask = None
    if config.get('mask_path', ''):
        mds = vu.load_mask(config['mask_path'], config['mask_key'], shape)
        mask = (mds[:] != 0).astype(np.uint8)
    nb = vu.Blocking([0, 0, 0], list(shape), block_shape).numberOfBlocks

    with _lib.Context(int(os.environ.get('CC_DEVICE', '0'))) as ctx:
        if fused:
            labels, res = ctx.label_volume(inp, block_shape, threshold, mode, mask)
            values = ctx.block_values(nb)
            lut = ctx.lut(res['n_labels'])
            np.save(os.path.join(tmp_folder, FUSED_LUT), lut)
            with open(os.path.join(tmp_folder, FUSED_MARKER), 'w') as f:
                json.dump({'output_path': os.path.abspath(config['output_path']),
                           'output_key': config['output_key'], 'n_labels': res['n_labels'],
                           'max_id': res['max_id'], 'n_components': res['n_components']}, f)
        else:
            x = torch.from_numpy(inp).cuda()
            m = None if mask is None else torch.from_numpy(mask).cuda()
            lab_dev, values = ctx.block_components(x, block_shape, threshold, mode, m)
            labels = lab_dev.cpu().numpy().view(np.uint64)
    with vu.file_reader(config['output_path']) as f:
        ds = f[config['output_key']]
        blocking = vu.Blocking([0, 0, 0], list(shape), block_shape)
        for b in block_list:           # empty blocks are not written (block_components.py:175-177)
            if values[b]:
                bb = vu.block_to_bb(blocking.getBlock(b))
                ds[bb] = labels[bb]
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
