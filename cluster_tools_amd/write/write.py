#! /usr/bin/python
"""Write task + job, dense-LUT path (reference: cluster_tools/write/write.py:29-131,157-220,249-387).
Per non-empty block: seg[seg != 0] += offset; seg = lut[seg] (cc_write on the device); job 0
sets attrs['maxId'] = lut.max().  When the labels were already produced by a fused
BlockComponents job, the relabel is skipped and only maxId and the logs are written.
The dict / pickled-map and label-multiset branches of the reference are out of scope."""
import json
import os
import sys

import numpy as np

from cluster_tools_amd.luigi_compat import Task, Parameter, TaskParameter
from cluster_tools_amd.cluster_tasks import LocalTask, DummyTask
import cluster_tools_amd.utils.volume_utils as vu
import cluster_tools_amd.utils.function_utils as fu


class WriteBase(Task):
    task_name = 'write'
    src_file = os.path.abspath(__file__)

    input_path = Parameter()
    input_key = Parameter()
    output_path = Parameter()
    output_key = Parameter()
    assignment_path = Parameter()
    assignment_key = Parameter(default=None)
    dependency = TaskParameter(default=DummyTask())
    identifier = Parameter()
    offset_path = Parameter(default='')

    def requires(self):
        return self.dependency

    @staticmethod
    def default_task_config():
        config = LocalTask.default_task_config()
        config.update({'chunks': None, 'allow_empty_assignments': False})
        return config

    def run_impl(self):
        shebang, block_shape, roi_begin, roi_end, block_list_path = self.global_config_values(True)
        self.init(shebang)
        with vu.file_reader(self.input_path, 'r') as f:
            shape = f[self.input_key].shape
        config = self.get_task_config()
        chunks = config.pop('chunks', None)
        if chunks is None:
            chunks = tuple(min(bs // 2, sh) for bs, sh in zip(block_shape, shape))
        with vu.file_reader(self.output_path) as f:
            if self.output_key in f:
                chunks = f[self.output_key].chunks
            assert all(bs % ch == 0 for bs, ch in zip(block_shape, chunks)), '%s, %s' % (str(block_shape), str(chunks))
            f.require_dataset(self.output_key, shape=shape, chunks=chunks, compression='gzip', dtype='uint64')
        in_place = self.input_path == self.output_path and self.input_key == self.output_key
        if self.assignment_key is None:
            raise NotImplementedError('pickled assignment maps are not supported on the MI355X path')
        config.update({'input_path': self.input_path, 'input_key': self.input_key, 'block_shape': block_shape,
                       'assignment_path': self.assignment_path, 'assignment_key': self.assignment_key,
                       'tmp_folder': self.tmp_folder})
        if self.offset_path != '':
            config.update({'offset_path': self.offset_path})
        if not in_place:
            config.update({'output_path': self.output_path, 'output_key': self.output_key})
        block_list = vu.blocks_in_volume(shape, block_shape, roi_begin, roi_end, block_list_path=block_list_path)
        self._write_log('scheduling %i blocks to be processed' % len(block_list))
        n_jobs = 1
        self.prepare_jobs(n_jobs, block_list, config, self.identifier)
        self.submit_jobs(n_jobs, self.identifier)
        self.wait_for_jobs(self.identifier)
        self.check_jobs(n_jobs, self.identifier)

    def output(self):
        from cluster_tools_amd.luigi_compat import LocalTarget
        return LocalTarget(os.path.join(self.tmp_folder, '%s_%s.log' % (self.task_name, self.identifier)))


class WriteLocal(WriteBase, LocalTask):
    pass


def write(job_id, config_path):
    from cluster_tools_amd.thresholded_components.block_faces import fused_run
    fu.log('start processing job %i' % job_id)
    fu.log('loading config from %s' % config_path)
    with open(config_path) as f:
        config = json.load(f)
    input_path, input_key = config['input_path'], config['input_key']
    output_path = config.get('output_path', input_path)
    output_key = config.get('output_key', input_key)
    block_shape, block_list = config['block_shape'], config['block_list']
    with vu.file_reader(config['assignment_path'], 'r') as f:
        lut = f[config['assignment_key']][:]
    offset_path = config.get('offset_path', None)
    if offset_path is not None:
        with open(offset_path) as f:
            od = json.load(f)
        offsets, empty_blocks = np.array(od['offsets'], dtype=np.uint64), set(od['empty_blocks'])
    else:
        offsets, empty_blocks = None, set()
    in_place = output_path == input_path and output_key == input_key
    done = in_place and offset_path is not None and fused_run(config.get('tmp_folder', ''), input_path, input_key)
    if done:
        fu.log('labels already final (fused BlockComponents job)')
    else:
        import torch
        from cluster_tools_amd import _lib
        with vu.file_reader(input_path, 'r') as f:
            seg = f[input_key][:]
        shape = seg.shape
        nb = vu.Blocking([0, 0, 0], list(shape), block_shape).numberOfBlocks
        offs = offsets if offsets is not None else np.zeros(nb, dtype=np.uint64)
        dev = torch.from_numpy(seg.view(np.int64)).cuda()
        with _lib.Context(int(os.environ.get('CC_DEVICE', '0'))) as ctx:
            ctx.write(dev, block_shape, offs, lut)
        seg = dev.cpu().numpy().view(np.uint64)
        blocking = vu.Blocking([0, 0, 0], list(shape), block_shape)
        with vu.file_reader(output_path) as f:
            ds = f[output_key]
            for b in block_list:
                if b in empty_blocks:
                    continue
                bb = vu.block_to_bb(blocking.getBlock(b))
                ds[bb] = seg[bb]
    for b in block_list:
        if b not in empty_blocks:
            fu.log_block_success(b)
    if job_id == 0:
        with vu.file_reader(output_path) as f:
            f[output_key].attrs['maxId'] = int(lut.max())
    fu.log_job_success(job_id)


if __name__ == '__main__':
    path = sys.argv[1]
    assert os.path.exists(path), path
    job_id = int(os.path.split(path)[1].split('.')[0].split('_')[-1])
    write(job_id, path)
