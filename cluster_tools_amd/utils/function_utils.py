"""stdout logging contract of the job scripts (cluster_tools/utils/function_utils.py:7-16):
LocalTask.check_jobs reads the last line of each job log and expects 'processed job <i>'."""
from datetime import datetime


def log(msg):
    print('%s: %s' % (str(datetime.now()), msg), flush=True)


def log_block_success(block_id):
    print('%s: processed block %i' % (str(datetime.now()), block_id), flush=True)


def log_job_success(job_id):
    print('%s: processed job %i' % (str(datetime.now()), job_id), flush=True)
