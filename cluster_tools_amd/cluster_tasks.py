"""Task / job framework of the reference, target='local' (cluster_tools/cluster_tasks.py:27-386,
515-555, 645-676), kept so the MI355X path is a drop-in for it:

  * configs: <config_dir>/global.config and <config_dir>/<task_name>.config (JSON), defaults
    from default_global_config() / default_task_config();
  * jobs: the task's module file is copied to <tmp>/<task_name>.py (shebang replaced) and run
    as `<tmp>/<task_name>.py <tmp>/<task_name>_job_<i>.config`, stdout to
    <tmp>/logs/<task_name>_<i>.log; a job succeeded iff its last log line is
    '<datetime>: processed job <i>';
  * target: <tmp>/<task_name>.log (moved to *_failed.log on failure); retries as the reference.

Only the local target exists here: Slurm / LSF are multi-node batch schedulers outside the
hot path.
"""
import json
import os
import shutil
import stat
import subprocess
import sys
import time
from concurrent import futures
from datetime import datetime
from multiprocessing import cpu_count

from .luigi_compat import Task, Parameter, IntParameter, TaskParameter, Target, LocalTarget
from .utils.parse_utils import parse_job, parse_blocks_task

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class FailedJobsError(Exception):
    pass


class DummyTarget(Target):
    def exists(self):
        return True


class DummyTask(Task):
    """cluster_tools/utils/task_utils.py:11-15"""

    def output(self):
        return DummyTarget()


class BaseClusterTask(Task):
    tmp_folder = Parameter()
    max_jobs = IntParameter()
    config_dir = Parameter()
    allow_retry = True
    n_retries = 0

    def run(self):
        self.make_dirs()
        self._write_log('Start task %s' % self.task_name)
        try:
            self.run_impl()
        except FailedJobsError:
            raise
        except Exception as e:
            out_path = self.output().path
            self._write_log('task failed in `run_impl` with %s' % str(e))
            shutil.move(out_path, out_path[:-4] + '_failed.log')
            raise
        self._write_log('Done task %s' % self.task_name)

    def init(self, shebang):
        self._write_script_file(shebang)

    @staticmethod
    def parse_jobs(log_prefix, max_jobs):
        return [j for j in range(max_jobs) if parse_job(log_prefix + '%i.log' % j, j)]

    def check_jobs(self, n_jobs, job_prefix=None):
        job_name = self.task_name if job_prefix is None else '%s_%s' % (self.task_name, job_prefix)
        log_prefix = os.path.join(self.tmp_folder, 'logs', '%s_' % job_name)
        success = self.parse_jobs(log_prefix, n_jobs)
        if len(success) == n_jobs:
            self._write_log('%s finished successfully' % self.task_name)
            return
        failed = sorted(set(range(n_jobs)) - set(success))
        self._write_log('%s failed for jobs:' % self.task_name)
        self._write_log(', '.join(map(str, failed)))
        max_num_retries = self.get_global_config().get('max_num_retries', 0)
        retry = self.n_retries < max_num_retries and self.allow_retry and len(failed) / n_jobs < 0.5
        if retry:
            passed = parse_blocks_task(log_prefix, n_jobs, success)
            self.block_list = sorted(set(self.block_list) - set(passed))
            self._write_log('resubmitting %i failed blocks in %i retry attempt' % (len(self.block_list),
                                                                                   self.n_retries + 1))
            self.n_retries += 1
            self.run()
        else:
            out_path = self.output().path
            shutil.move(out_path, out_path[:-4] + '_failed.log')
            raise FailedJobsError('Task: %s failed for %i / %i jobs' % (self.task_name, len(failed), n_jobs))

    def get_task_config(self):
        path = os.path.join(self.config_dir, self.task_name + '.config')
        if os.path.exists(path):
            self._write_log('reading task config from %s' % path)
            with open(path) as f:
                return json.load(f)
        self._write_log('reading default task config')
        return self.default_task_config()

    @staticmethod
    def default_task_config():
        return {'threads_per_job': 1, 'time_limit': 60, 'mem_limit': 1., 'qos': 'normal',
                'slurm_requirements': []}

    def get_global_config(self):
        path = os.path.join(self.config_dir, 'global.config')
        if os.path.exists(path):
            with open(path) as f:
                return json.load(f)
        return self.default_global_config()

    @staticmethod
    def default_global_config():
        return {'block_shape': [50, 512, 512], 'shebang': sys.executable, 'roi_begin': None,
                'roi_end': None, 'groupname': None, 'partition': None, 'max_num_retries': 0,
                'block_list_path': None, 'easybuild': True, 'qos': 'normal'}

    def global_config_values(self, with_block_list_path=False):
        config = self.get_global_config()
        conf = (config['shebang'], config['block_shape'], config.get('roi_begin', None),
                config.get('roi_end', None))
        if with_block_list_path:
            conf = conf + (config.get('block_list_path', None),)
        return conf

    def output(self):
        return LocalTarget(os.path.join(self.tmp_folder, self.task_name + '.log'))

    # ---- helpers ----
    def _write_log(self, msg):
        with open(self.output().path, 'a') as f:
            f.write('%s: %s\n' % (str(datetime.now()), msg))

    def _config_path(self, job_id, job_prefix=None):
        if job_prefix is None:
            return os.path.join(self.tmp_folder, self.task_name + '_job_%s.config' % str(job_id))
        return os.path.join(self.tmp_folder, self.task_name + '_job_%s_%s.config' % (job_prefix, str(job_id)))

    def make_dirs(self):
        os.makedirs(self.tmp_folder, exist_ok=True)
        os.makedirs(os.path.join(self.tmp_folder, 'logs'), exist_ok=True)
        os.makedirs(os.path.join(self.tmp_folder, 'error_logs'), exist_ok=True)
        self._write_log('created tmp-folder and log dirs @ %s' % self.tmp_folder)

    def _write_job_config(self, n_jobs, block_list, config, job_prefix=None, consecutive_blocks=False):
        if block_list is None:
            assert n_jobs == 1
            with open(self._config_path(0, job_prefix), 'w') as f:
                json.dump(config, f)
        else:
            self.block_list = block_list
            for job_id in range(n_jobs):
                job_config = {'block_list': block_list[job_id::n_jobs], **config}
                with open(self._config_path(job_id, job_prefix), 'w') as f:
                    json.dump(job_config, f)
        self._write_log('written config for %i jobs' % n_jobs)

    def _write_script_file(self, shebang):
        trgt = os.path.join(self.tmp_folder, self.task_name + '.py')
        shutil.copy(self.src_file, trgt)
        executable = shebang[2:].strip() if shebang.startswith('#!') else shebang
        if not os.path.exists(executable):
            raise RuntimeError('The python executable %s is not valid' % executable)
        with open(trgt) as f:
            lines = f.read().split('\n')
        lines[0] = '#! ' + executable
        with open(trgt, 'w') as f:
            f.write('\n'.join(lines))
        os.chmod(trgt, os.stat(trgt).st_mode | stat.S_IEXEC)
        self._write_log('copied python script from %s to %s' % (self.src_file, trgt))


class LocalTask(BaseClusterTask):
    max_local_jobs = cpu_count()

    def prepare_jobs(self, n_jobs, block_list, config, job_prefix=None, consecutive_blocks=False):
        self._write_job_config(n_jobs, block_list, config, job_prefix, consecutive_blocks)

    def _submit(self, job_id, job_prefix):
        script = os.path.join(self.tmp_folder, self.task_name + '.py')
        config_file = self._config_path(job_id, job_prefix)
        job_name = self.task_name if job_prefix is None else '%s_%s' % (self.task_name, job_prefix)
        log_file = os.path.join(self.tmp_folder, 'logs', '%s_%i.log' % (job_name, job_id))
        err_file = os.path.join(self.tmp_folder, 'error_logs', '%s_%i.err' % (job_name, job_id))
        env = dict(os.environ)
        env['PYTHONPATH'] = _REPO + (os.pathsep + env['PYTHONPATH'] if env.get('PYTHONPATH') else '')
        t0 = time.perf_counter()
        with open(log_file, 'w') as fo, open(err_file, 'w') as fe:
            subprocess.call([script, config_file], stdout=fo, stderr=fe, env=env)
        self._write_log('job %s %i wall %.3f s' % (job_name, job_id, time.perf_counter() - t0))

    def submit_jobs(self, n_jobs, job_prefix=None):
        assert n_jobs <= self.max_local_jobs
        with futures.ThreadPoolExecutor(n_jobs) as tp:
            list(tp.map(lambda j: self._submit(j, job_prefix), range(n_jobs)))

    def wait_for_jobs(self, job_prefix=None):
        pass


class WorkflowBase(Task):
    tmp_folder = Parameter()
    max_jobs = IntParameter()
    config_dir = Parameter()
    target = Parameter()
    dependency = TaskParameter(default=DummyTask())

    _target_dict = {'local': 'Local'}

    def _get_task_name(self, task_base_name):
        t = self.target.lower()
        if t not in self._target_dict:
            raise NotImplementedError("target '%s': only 'local' is available on the MI355X path" % self.target)
        return task_base_name + self._target_dict[t]

    def output(self):
        return LocalTarget(self.input().path)

    @staticmethod
    def get_config():
        return {'global': BaseClusterTask.default_global_config()}
