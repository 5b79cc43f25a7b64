#! /usr/bin/python
"""MergeAssignments task + job (reference: cluster_tools/thresholded_components/merge_assignments.py).
Union-find over ids 0..n_labels-1 (cc_merge_assignments, representative = smallest id) and the
1-D uint64 'assignments' dataset (chunks min(65334, n_labels), gzip).

By default all face pairs are merged.  The reference drops every merge when one block_faces job
saved an empty pair file (merge_assignments.py:115-123 with block_faces.py:169-176; SURVEY.md
§0.4); the task config key 'reference_empty_job_quirk' (default False) reproduces that branch for
this run's max_jobs: face job j owns blocks j :: min(n_blocks, max_jobs) (cluster_tasks.py:331),
and if any of them has no block with an upper-face pair the LUT is the identity.  The fused
BlockComponents job applies the same rule on the device (CC_OPT_EMPTY_JOB_QUIRK)."""
import json
import os
import sys

import numpy as np

from cluster_tools_amd.luigi_compat import Task, Parameter, ListParameter, TaskParameter
from cluster_tools_amd.cluster_tasks import LocalTask
import cluster_tools_amd.utils.volume_utils as vu
import cluster_tools_amd.utils.function_utils as fu
from cluster_tools_amd.thresholded_components.block_components import FUSED_MARKER, FUSED_LUT


QUIRK_KEY = 'reference_empty_job_quirk'
FACE_FLAGS = 'cc_face_blocks.npy'       # per block: 1 if it has an upper-face pair (BlockFaces job)


def any_empty_job(block_has_pairs, max_jobs):
    """Would one of the reference's block_faces jobs save an empty file?  Jobs own the blocks
    j :: n_jobs with n_jobs = min(n_blocks, max_jobs) (cluster_tasks.py:301-335)."""
    flags = np.asarray(block_has_pairs) != 0
    n_jobs = max(1, min(len(flags), int(max_jobs)))
    return any(not flags[j::n_jobs].any() for j in range(n_jobs))


class MergeAssignmentsBase(Task):
    task_name = 'merge_assignments'
    src_file = os.path.abspath(__file__)
    allow_retry = False

    output_path = Parameter()
    output_key = Parameter()
    shape = ListParameter()
    offset_path = Parameter()
    save_prefix = Parameter(default='cc_assignments')
    dependency = TaskParameter()

    def requires(self):
        return self.dependency

    def run_impl(self):
        shebang, block_shape, roi_begin, roi_end = self.global_config_values()
        self.init(shebang)
        config = self.get_task_config()
        config.update({'output_path': self.output_path, 'output_key': self.output_key,
                       'tmp_folder': self.tmp_folder, 'n_jobs': 1, 'offset_path': self.offset_path,
                       'save_prefix': self.save_prefix, 'max_jobs': int(self.max_jobs)})
        self.prepare_jobs(1, None, config)
        self.submit_jobs(1)
        self.wait_for_jobs()
        self.check_jobs(1)


class MergeAssignmentsLocal(MergeAssignmentsBase, LocalTask):
    pass


def merge_assignments(job_id, config_path):
    fu.log('start processing job %i' % job_id)
    fu.log('reading config from %s' % config_path)
    with open(config_path) as f:
        config = json.load(f)
    tmp_folder = config['tmp_folder']
    with open(config['offset_path']) as f:
        n_labels = int(json.load(f)['n_labels'])
    fused = os.path.join(tmp_folder, FUSED_MARKER)
    if os.path.exists(fused):
        lut = np.load(os.path.join(tmp_folder, FUSED_LUT))
        assert len(lut) == n_labels, (len(lut), n_labels)
        fu.log('assignments from the fused BlockComponents job')
    else:
        from cluster_tools_amd import _lib
        pairs = [np.load(os.path.join(tmp_folder, '%s_%i.npy' % (config['save_prefix'], j)))
                 for j in range(config['n_jobs'])]
        pairs = [p.reshape(-1, 2) for p in pairs if p.size]
        pairs = np.concatenate(pairs, axis=0).astype(np.uint64) if pairs else np.zeros((0, 2), np.uint64)
        fu.log('have %i pairs of node assignments' % len(pairs))
        flags_path = os.path.join(tmp_folder, FACE_FLAGS)
        if config.get(QUIRK_KEY, False) and os.path.exists(flags_path) and \
                any_empty_job(np.load(flags_path), config['max_jobs']):
            fu.log('a block_faces job of %i has no pairs: no merge (reference empty-job branch)'
                   % min(len(np.load(flags_path)), config['max_jobs']))
            lut = np.arange(n_labels, dtype=np.uint64)
        else:
            with _lib.Context(int(os.environ.get('CC_DEVICE', '0'))) as ctx:
                lut = ctx.merge_assignments(pairs, n_labels)
    chunks = (min(65334, n_labels),)
    with vu.file_reader(config['output_path']) as f:
        f.create_dataset(config['output_key'], data=lut, compression='gzip', chunks=chunks)
    fu.log_job_success(job_id)


if __name__ == '__main__':
    path = sys.argv[1]
    assert os.path.exists(path), path
    job_id = int(os.path.split(path)[1].split('.')[0].split('_')[-1])
    merge_assignments(job_id, path)
