#! /usr/bin/python
"""Threshold task + job (reference: cluster_tools/thresholded_components/threshold.py).

Same task surface as the reference (threshold.py:17-105): parameters input_path / input_key /
output_path / output_key / threshold / threshold_mode / channel / dependency, the task config
(sigma_prefilter, chunks, compression), the uint8 output dataset with chunks block_shape // 2
clipped to the shape, the job config per LocalTask and the "processed job" log contract.  The
job's compute (per-block normalize + float32 compare, threshold.py:131-171) runs on the MI355X
through cc_threshold (k_block_stats -> k_block_params -> k_threshold); one GPU job thresholds
the whole volume and writes the listed blocks.  channel (4-D input): the listed channels are
averaged on the device first (cc_channel_mean, threshold.py:139-148); sigma_prefilter > 0: per block
normalize + Gaussian smoothing first (cc_gaussian_smooth_blocks, threshold.py:150-153).
"""
import json
import os

import numpy as np

from cluster_tools_amd.luigi_compat import Task, Parameter, FloatParameter, TaskParameter
from cluster_tools_amd.cluster_tasks import LocalTask, DummyTask
import cluster_tools_amd.utils.volume_utils as vu
import cluster_tools_amd.utils.function_utils as fu


class ThresholdBase(Task):
    task_name = 'threshold'
    src_file = os.path.abspath(__file__)
    allow_retry = False

    input_path = Parameter()
    input_key = Parameter()
    output_path = Parameter()
    output_key = Parameter()
    threshold = FloatParameter()
    threshold_mode = Parameter(default='greater')
    channel = Parameter(default=None)
    dependency = TaskParameter(default=DummyTask())

    threshold_modes = ('greater', 'less', 'equal')

    @staticmethod
    def default_task_config():
        config = LocalTask.default_task_config()
        config.update({'sigma_prefilter': 0})
        return config

    def requires(self):
        return self.dependency

    def run_impl(self):
        shebang, block_shape, roi_begin, roi_end, block_list_path = \
            self.global_config_values(with_block_list_path=True)
        self.init(shebang)
        shape = vu.get_shape(self.input_path, self.input_key)
        assert self.threshold_mode in self.threshold_modes
        config = self.get_task_config()
        config.update({'input_path': self.input_path, 'input_key': self.input_key,
                       'output_path': self.output_path, 'output_key': self.output_key,
                       'block_shape': block_shape, 'threshold': self.threshold,
                       'threshold_mode': self.threshold_mode})
        chunks = config.pop('chunks', None)
        if chunks is None:
            chunks = tuple(bs // 2 for bs in block_shape)
        if self.channel is None:
            assert len(shape) == 3, str(len(shape))
        else:
            assert len(shape) == 4, str(len(shape))
            from cluster_tools_amd.thresholded_components.block_components import channel_list
            assert all(0 <= c < shape[0] for c in channel_list(self.channel)), (shape[0], self.channel)
            shape = shape[1:]
            config.update({'channel': self.channel})
        chunks = tuple(max(1, min(ch, sh)) for ch, sh in zip(chunks, shape))
        compression = config.pop('compression', 'gzip')
        with vu.file_reader(self.output_path) as f:
            f.require_dataset(self.output_key, shape=shape, dtype='uint8', compression=compression, chunks=chunks)
        block_list = vu.blocks_in_volume(shape, block_shape, roi_begin, roi_end)
        n_jobs = 1                     # one GPU job thresholds the volume
        self.prepare_jobs(n_jobs, block_list, config)
        self.submit_jobs(n_jobs)
        self.wait_for_jobs()
        self.check_jobs(n_jobs)


class ThresholdLocal(ThresholdBase, LocalTask):
    pass


def threshold(job_id, config_path):
    import torch
    from cluster_tools_amd import _lib
    fu.log('start processing job %i' % job_id)
    fu.log('reading config from %s' % config_path)
    with open(config_path) as f:
        config = json.load(f)
    block_list = config['block_list']
    block_shape = config['block_shape']
    thr, mode = config['threshold'], config['threshold_mode']
    fu.log('Applying threshold %f with mode %s' % (thr, mode))
    from cluster_tools_amd.thresholded_components.block_components import read_input, to_device
    inp, chans = read_input(config)
    shape = inp.shape if chans is None else inp.shape[1:]
    with _lib.Context(int(os.environ.get('CC_DEVICE', '0'))) as ctx:
        x = to_device(ctx, inp, chans, ctx.torch_device(), config)
        out = ctx.threshold(x, block_shape, thr, mode).cpu().numpy()
    blocking = vu.Blocking([0, 0, 0], list(shape), block_shape)
    with vu.file_reader(config['output_path']) as f:
        ds = f[config['output_key']]
        for b in block_list:
            bb = vu.block_to_bb(blocking.getBlock(b))
            ds[bb] = out[bb]
            fu.log_block_success(b)
    fu.log_job_success(job_id)


if __name__ == '__main__':
    import sys
    path = sys.argv[1]
    assert os.path.exists(path), path
    job_id = int(os.path.split(path)[1].split('.')[0].split('_')[-1])
    threshold(job_id, path)
