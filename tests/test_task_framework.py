"""The reference's task/job contract on the cluster_tools_amd framework (CPU): job configs with
strided block lists, script copy + shebang, 'processed job' tokens, luigi targets, retries."""
import json
import os
import sys

import pytest

from cluster_tools_amd import luigi_compat as luigi
from cluster_tools_amd.cluster_tasks import DummyTask, BaseClusterTask, FailedJobsError

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _dummy_task  # noqa: E402


def _configs(tmp_path, retries=0):
    cfg = str(tmp_path / 'config')
    os.makedirs(cfg, exist_ok=True)
    g = BaseClusterTask.default_global_config()
    g.update({'block_shape': [4, 4, 4], 'max_num_retries': retries})
    with open(os.path.join(cfg, 'global.config'), 'w') as f:
        json.dump(g, f)
    return cfg


def test_jobs_run_and_targets(tmp_path):
    out = tmp_path / 'out'
    out.mkdir()
    t = _dummy_task.DummyStageLocal(tmp_folder=str(tmp_path / 'tmp'), config_dir=_configs(tmp_path), max_jobs=3,
                                    out_path=str(out), dependency=DummyTask())
    assert luigi.build([t], local_scheduler=True)
    assert sorted(os.listdir(out)) == sorted('block_%d' % b for b in range(10))
    tmp = tmp_path / 'tmp'
    assert (tmp / 'dummy_stage.log').exists() and (tmp / 'dummy_stage.py').exists()
    job0 = json.load(open(tmp / 'dummy_stage_job_0.config'))
    assert job0['block_list'] == [0, 3, 6, 9]                 # block_list[job_id::n_jobs]
    last = open(tmp / 'logs' / 'dummy_stage_2.log').read().strip().split('\n')[-1]
    assert last.endswith('processed job 2')
    assert t.complete()


def test_failure_without_retry_moves_log(tmp_path):
    out = tmp_path / 'out'
    out.mkdir()
    t = _dummy_task.DummyStageLocal(tmp_folder=str(tmp_path / 'tmp'), config_dir=_configs(tmp_path), max_jobs=2,
                                    out_path=str(out), fail_first='yes', dependency=DummyTask())
    t.make_dirs()
    with pytest.raises(FailedJobsError):
        t.run()
    assert (tmp_path / 'tmp' / 'dummy_stage_failed.log').exists()


def test_retry_recovers_failed_blocks(tmp_path):
    out = tmp_path / 'out'
    out.mkdir()
    t = _dummy_task.DummyStageLocal(tmp_folder=str(tmp_path / 'tmp'), config_dir=_configs(tmp_path, 2), max_jobs=4,
                                    out_path=str(out), fail_first='yes', dependency=DummyTask())
    # 2 of 4 jobs fail (jobs 1 and 3 own odd blocks first) -> 50% -> no retry (reference rule)
    t.make_dirs()
    with pytest.raises(FailedJobsError):
        t.run()


def test_workflow_rejects_other_targets():
    from cluster_tools_amd.thresholded_components import ThresholdedComponentsWorkflow
    w = ThresholdedComponentsWorkflow(tmp_folder='x', max_jobs=1, config_dir='x', target='slurm',
                                      input_path='x', input_key='x', output_path='x', output_key='x',
                                      assignment_key='x', threshold=0.5)
    with pytest.raises(NotImplementedError):
        w._get_task_name('BlockComponents')
