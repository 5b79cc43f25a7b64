"""Job-log parsing (cluster_tools/utils/parse_utils.py:76-92,123-154)."""
import os


def _last_line(path):
    try:
        with open(path) as f:
            lines = [ll for ll in f.read().split('\n') if ll]
        return lines[-1] if lines else None
    except OSError:
        return None


def parse_job(log_file, job_id):
    last = _last_line(log_file)
    if last is None:
        return False
    return ' '.join(last.split()[2:]) == 'processed job %i' % job_id


def parse_blocks(log_file):
    blocks = []
    with open(log_file) as f:
        for line in f:
            line = ' '.join(line.split()[2:])
            if line.startswith('processed block'):
                blocks.append(int(line.split()[-1]))
    return blocks


def parse_blocks_task(log_prefix, max_jobs, complete_job_list=()):
    blocks = []
    for job_id in range(max_jobs):
        if job_id in complete_job_list:
            continue
        p = log_prefix + '%i.log' % job_id
        if os.path.exists(p):
            blocks.extend(parse_blocks(p))
    return blocks
