#! /usr/bin/python
"""BlockFaces task + job (reference: cluster_tools/thresholded_components/block_faces.py:21-177).
Face pairs (label_a + off_a, label_b + off_b) of every block's upper faces, deduplicated, saved
as <tmp>/cc_assignments_<job>.npy; computed by cc_block_faces on the device.  After a fused
BlockComponents job the merge is already done, and the job only logs."""
import json
import os
import sys

import numpy as np

from cluster_tools_amd.luigi_compat import Task, Parameter, TaskParameter
from cluster_tools_amd.cluster_tasks import LocalTask
import cluster_tools_amd.utils.volume_utils as vu
import cluster_tools_amd.utils.function_utils as fu
from cluster_tools_amd.thresholded_components.block_components import FUSED_MARKER


class BlockFacesBase(Task):
    task_name = 'block_faces'
    src_file = os.path.abspath(__file__)
    allow_retry = False

    input_path = Parameter()
    input_key = Parameter()
    offsets_path = Parameter()
    dependency = TaskParameter()

    def requires(self):
        return self.dependency

    def run_impl(self):
        shebang, block_shape, roi_begin, roi_end = self.global_config_values()
        self.init(shebang)
        shape = vu.get_shape(self.input_path, self.input_key)
        config = self.get_task_config()
        config.update({'input_path': self.input_path, 'input_key': self.input_key,
                       'offsets_path': self.offsets_path, 'block_shape': block_shape,
                       'tmp_folder': self.tmp_folder})
        block_list = vu.blocks_in_volume(shape, block_shape, roi_begin, roi_end)
        n_jobs = 1
        self.prepare_jobs(n_jobs, block_list, config)
        self.submit_jobs(n_jobs)
        self.wait_for_jobs()
        self.check_jobs(n_jobs)


class BlockFacesLocal(BlockFacesBase, LocalTask):
    pass


def fused_run(tmp_folder, path, key):
    """The fused marker of this tmp folder, if it covers dataset path/key."""
    m = os.path.join(tmp_folder, FUSED_MARKER)
    if not os.path.exists(m):
        return None
    with open(m) as f:
        info = json.load(f)
    if info['output_path'] == os.path.abspath(path) and info['output_key'] == key:
        return info
    return None


def block_faces(job_id, config_path):
    fu.log('start processing job %i' % job_id)
    fu.log('reading config from %s' % config_path)
    with open(config_path) as f:
        config = json.load(f)
    tmp_folder = config['tmp_folder']
    block_list = config['block_list']
    with open(config['offsets_path']) as f:
        od = json.load(f)
    offsets, n_labels = np.array(od['offsets'], dtype=np.uint64), od['n_labels']
    if fused_run(tmp_folder, config['input_path'], config['input_key']) is not None:
        fu.log('labels were merged by the fused BlockComponents job')
    else:
        import torch
        from cluster_tools_amd import _lib
        with vu.file_reader(config['input_path'], 'r') as f:
            seg = f[config['input_key']][:]
        from cluster_tools_amd.thresholded_components.merge_assignments import FACE_FLAGS
        with _lib.Context(int(os.environ.get('CC_DEVICE', '0'))) as ctx:
            pairs, flags = ctx.block_faces(torch.from_numpy(seg.view(np.int64)).cuda(), config['block_shape'],
                                           offsets, with_block_flags=True)
        if len(pairs):
            assert int(pairs.max()) < n_labels, '%i, %i' % (int(pairs.max()), n_labels)
        np.save(os.path.join(tmp_folder, 'cc_assignments_%i.npy' % job_id), pairs)
        # which blocks contribute pairs: the reference's per-job files are empty exactly when none
        # of a job's blocks does (merge_assignments.any_empty_job)
        np.save(os.path.join(tmp_folder, FACE_FLAGS), flags)
    for b in block_list:
        fu.log_block_success(b)
    fu.log_job_success(job_id)


if __name__ == '__main__':
    path = sys.argv[1]
    assert os.path.exists(path), path
    job_id = int(os.path.split(path)[1].split('.')[0].split('_')[-1])
    block_faces(job_id, path)
