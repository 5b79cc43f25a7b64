#! /usr/bin/python
"""MergeOffsets task + job (reference: cluster_tools/thresholded_components/merge_offsets.py:22-131).
Same inputs (per-job JSONs), same cc_offsets.json; the scan runs through cc_merge_offsets."""
import json
import os
import sys

import numpy as np

from cluster_tools_amd.luigi_compat import Task, Parameter, ListParameter, TaskParameter
from cluster_tools_amd.cluster_tasks import LocalTask
import cluster_tools_amd.utils.volume_utils as vu
import cluster_tools_amd.utils.function_utils as fu


class MergeOffsetsBase(Task):
    task_name = 'merge_offsets'
    src_file = os.path.abspath(__file__)
    allow_retry = False

    shape = ListParameter()
    save_path = Parameter()
    save_prefix = Parameter(default='connected_components_offsets')
    dependency = TaskParameter()

    def requires(self):
        return self.dependency

    def run_impl(self):
        shebang, block_shape, roi_begin, roi_end = self.global_config_values()
        self.init(shebang)
        block_list = vu.blocks_in_volume(self.shape, block_shape, roi_begin, roi_end)
        n_jobs = 1     # BlockComponents writes one JSON per (GPU) job
        config = self.get_task_config()
        config.update({'tmp_folder': self.tmp_folder, 'n_jobs': n_jobs, 'save_path': self.save_path,
                       'n_blocks': len(block_list), 'save_prefix': self.save_prefix})
        self.prepare_jobs(1, None, config)
        self.submit_jobs(1)
        self.wait_for_jobs()
        self.check_jobs(1)


class MergeOffsetsLocal(MergeOffsetsBase, LocalTask):
    pass


def merge_offsets(job_id, config_path):
    from cluster_tools_amd import _lib
    _lib.load(host_only=True)         # a one-shot job process: host arithmetic only, no torch import
    fu.log('start processing job %i' % job_id)
    fu.log('reading config from %s' % config_path)
    with open(config_path) as f:
        config = json.load(f)
    tmp_folder, n_jobs = config['tmp_folder'], config['n_jobs']
    n_blocks, save_prefix = config['n_blocks'], config['save_prefix']
    offsets = {}
    for block_job_id in range(n_jobs):
        path = os.path.join(tmp_folder, '%s_%i.json' % (save_prefix, block_job_id))
        with open(path) as f:
            offsets.update(json.load(f))
        os.remove(path)
    blocks = list(map(int, offsets.keys()))
    values = list(offsets.values())
    assert len(blocks) == len(values) == n_blocks
    key_sort = np.argsort(blocks)
    values = np.array([values[k] for k in key_sort], dtype='uint64')
    offs, empty_blocks, n_labels = _lib.merge_offsets(values)
    fu.log('number of empty blocks: %i / %i' % (len(empty_blocks), n_blocks))
    fu.log('total number of labels: %i' % n_labels)
    with open(config['save_path'], 'w') as f:
        json.dump({'offsets': [int(o) for o in offs], 'empty_blocks': [int(e) for e in empty_blocks],
                   'n_labels': int(n_labels)}, f)
    fu.log_job_success(job_id)


if __name__ == '__main__':
    path = sys.argv[1]
    assert os.path.exists(path), path
    job_id = int(os.path.split(path)[1].split('.')[0].split('_')[-1])
    merge_offsets(job_id, path)
