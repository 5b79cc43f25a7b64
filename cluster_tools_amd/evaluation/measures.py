#! /usr/bin/python
"""Measures task + job (reference: cluster_tools/evaluation/measures.py).

Same task surface as the reference MeasuresBase (measures.py:23-56: task_name 'measures', one
job, output_path JSON with 'vi-split', 'vi-merge', 'adapted-rand-error', 'rand-index').  The
reference reads the overlaps NodeLabelWorkflow serialized (node_labels/block_node_labels.py:
133-166 + merge_node_labels.py); here the one GPU job reads the segmentation and ground truth
and cc_evaluate computes the same overlaps (block grid of the global config, ws.sum() == 0 block
skip, gt ignore label) and the contingency-table measures on the MI355X in one pass
(cluster_tools_amd/csrc/cc_eval.hip).  Parameters are therefore seg / gt datasets instead of
input_path / overlap_key.
"""
import json
import os

import numpy as np

from cluster_tools_amd.luigi_compat import Task, Parameter, TaskParameter, BoolParameter
from cluster_tools_amd.cluster_tasks import LocalTask, DummyTask
import cluster_tools_amd.utils.volume_utils as vu
import cluster_tools_amd.utils.function_utils as fu


class MeasuresBase(Task):
    task_name = 'measures'
    src_file = os.path.abspath(__file__)
    allow_retry = False

    seg_path = Parameter()
    seg_key = Parameter()
    gt_path = Parameter()
    gt_key = Parameter()
    output_path = Parameter()
    ignore_label = BoolParameter(default=True)
    dependency = TaskParameter(default=DummyTask())

    def requires(self):
        return self.dependency

    def run_impl(self):
        shebang, block_shape, roi_begin, roi_end = self.global_config_values()
        self.init(shebang)
        config = self.get_task_config()
        shape = vu.get_shape(self.seg_path, self.seg_key)
        assert tuple(shape) == tuple(vu.get_shape(self.gt_path, self.gt_key)), 'seg / gt shapes differ'
        assert len(shape) == 3, str(len(shape))
        config.update({'seg_path': self.seg_path, 'seg_key': self.seg_key, 'gt_path': self.gt_path,
                       'gt_key': self.gt_key, 'output_path': self.output_path,
                       'ignore_label': 0 if self.ignore_label else None, 'block_shape': block_shape})
        n_jobs = 1
        self.prepare_jobs(n_jobs, None, config)
        self.submit_jobs(n_jobs)
        self.wait_for_jobs()
        self.check_jobs(n_jobs)


class MeasuresLocal(MeasuresBase, LocalTask):
    pass


def _read_u64(path, key):
    with vu.file_reader(path, 'r') as f:
        a = f[key][:]
    if a.dtype.kind not in 'ui':
        raise ValueError('%s/%s: integer labels expected, got %s' % (path, key, a.dtype))
    return np.ascontiguousarray(a.astype(np.uint64, copy=False))


def measures(job_id, config_path):
    import torch
    from cluster_tools_amd import _lib
    fu.log('start processing job %i' % job_id)
    fu.log('reading config from %s' % config_path)
    with open(config_path) as f:
        config = json.load(f)
    seg = _read_u64(config['seg_path'], config['seg_key'])
    gt = _read_u64(config['gt_path'], config['gt_key'])
    with _lib.Context(int(os.environ.get('CC_DEVICE', '0'))) as ctx:
        r = ctx.evaluate(torch.from_numpy(seg.view(np.int64)).cuda(), torch.from_numpy(gt.view(np.int64)).cuda(),
                         config['block_shape'], ignore_label=config['ignore_label'])
    fu.log('contingency table: %i pairs over %i points' % (r['n_pairs'], r['n_points']))
    results = {'vi-split': r['vi_split'], 'vi-merge': r['vi_merge'],
               'adapted-rand-error': r['adapted_rand_error'], 'rand-index': r['rand_index']}
    with open(config['output_path'], 'w') as f:
        json.dump(results, f)
    fu.log_job_success(job_id)


if __name__ == '__main__':
    import sys
    path = sys.argv[1]
    assert os.path.exists(path), path
    job_id = int(os.path.split(path)[1].split('.')[0].split('_')[-1])
    measures(job_id, path)
