#! /usr/bin/python
"""A trivial task on the cluster_tools_amd LocalTask framework (tests/test_task_framework.py)."""
import json
import os
import sys

from cluster_tools_amd.luigi_compat import Task, Parameter, TaskParameter
from cluster_tools_amd.cluster_tasks import LocalTask
import cluster_tools_amd.utils.function_utils as fu


class DummyStageBase(Task):
    task_name = 'dummy_stage'
    src_file = os.path.abspath(__file__)
    allow_retry = True
    out_path = Parameter()
    fail_first = Parameter(default='')
    dependency = TaskParameter()

    def requires(self):
        return self.dependency

    def run_impl(self):
        shebang, block_shape, roi_begin, roi_end = self.global_config_values()
        self.init(shebang)
        config = self.get_task_config()
        config.update({'out_path': self.out_path, 'fail_first': self.fail_first, 'tmp_folder': self.tmp_folder})
        n_jobs = min(4, self.max_jobs)
        self.prepare_jobs(n_jobs, list(range(10)), config)
        self.submit_jobs(n_jobs)
        self.wait_for_jobs()
        self.check_jobs(n_jobs)


class DummyStageLocal(DummyStageBase, LocalTask):
    pass


def dummy_stage(job_id, config_path):
    with open(config_path) as f:
        config = json.load(f)
    marker = os.path.join(config['tmp_folder'], 'failed_once_%d' % job_id)
    for b in config['block_list']:
        # fault injection like test/retry/failing_task.py:72-78: odd blocks fail on the first try
        if config['fail_first'] and b % 2 == 1 and not os.path.exists(marker):
            open(marker, 'w').close()
            raise RuntimeError('injected failure')
        with open(os.path.join(config['out_path'], 'block_%d' % b), 'w') as f:
            f.write('1')
        fu.log_block_success(b)
    fu.log_job_success(job_id)


if __name__ == '__main__':
    path = sys.argv[1]
    job_id = int(os.path.split(path)[1].split('.')[0].split('_')[-1])
    dummy_stage(job_id, path)
