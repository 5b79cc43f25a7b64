"""BASELINE config 1 through the drop-in API, with the wall-clock split.

    python tools/bench_c1.py [--mode greater] [--repeats 2] [--out DIR]

Writes a CREMI-sized (125, 1250, 1250) float32 boundary map (synthetic: the CREMI sample is not
available) as a gzip N5 dataset, runs ThresholdedComponentsWorkflow(target='local', threshold 0.5,
block_shape [50, 512, 512] = the reference default, max_jobs 16) and prints one JSON line: the
workflow wall time, each stage job's process wall, the fused job's n5-read /
H2D+device+D2H (cc_label_volume_host, no torch in the job) / n5-write split (<tmp>/cc_fused_timing.json), and the C restatement of the reference path (oracle/cc_oracle.c,
in memory, no gzip) on the same voxels and the same host threads.  Run on the GPU box.
"""
import argparse
import json
import os
import re
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--mode', default='greater')
    p.add_argument('--repeats', type=int, default=2)
    p.add_argument('--out', default=None)
    a = p.parse_args()
    import numpy as np
    from cluster_tools_amd import _lib, n5
    from cluster_tools_amd import luigi_compat as luigi
    from cluster_tools_amd.cluster_tasks import BaseClusterTask
    from cluster_tools_amd.thresholded_components import ThresholdedComponentsWorkflow
    from oracle import oracle as O

    _lib.check_provenance()
    shape, bs = (125, 1250, 1250), [50, 512, 512]
    work = a.out or tempfile.mkdtemp(prefix='cc_c1_')
    os.makedirs(work, exist_ok=True)
    with _lib.Context(0) as ctx:
        x = ctx.generate_boundary_map(shape).cpu().numpy()
    data = os.path.join(work, 'c1.n5')
    t = time.perf_counter()
    with n5.open_file(data) as f:
        f.create_dataset('volumes/raw/boundaries', data=x, chunks=(25, 256, 256), compression='gzip')
    t_in = time.perf_counter() - t
    cfg = os.path.join(work, 'config')
    os.makedirs(cfg, exist_ok=True)
    g = BaseClusterTask.default_global_config()
    with open(os.path.join(cfg, 'global.config'), 'w') as f:
        json.dump(g, f)
    runs = []
    for r in range(a.repeats):
        tmp = os.path.join(work, 'tmp%d' % r)
        key = 'segmentation/cc%d' % r
        wf = ThresholdedComponentsWorkflow(tmp_folder=tmp, config_dir=cfg, target='local', max_jobs=16,
                                           input_path=data, input_key='volumes/raw/boundaries', output_path=data,
                                           output_key=key, assignment_key='segmentation/assignments%d' % r,
                                           threshold=0.5, threshold_mode=a.mode)
        t = time.perf_counter()
        assert luigi.build([wf], local_scheduler=True)
        wall = time.perf_counter() - t
        with open(os.path.join(tmp, 'cc_fused_timing.json')) as f:
            timing = json.load(f)
        # per-stage job wall (cluster_tasks.LocalTask._submit logs each job process's wall time)
        jobs = {}
        for fn in sorted(os.listdir(tmp)):
            if fn.endswith('.log'):
                for m in re.finditer(r'job (\S+) (\d+) wall ([\d.]+) s', open(os.path.join(tmp, fn)).read()):
                    jobs[m.group(1)] = float(m.group(3))
        runs.append({'workflow_wall_s': round(wall, 3), 'job_wall_s': jobs,
                     **{k: round(v, 4) if isinstance(v, float) else v for k, v in timing.items()}})
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    t = time.perf_counter()
    ref = O.label_volume(x, bs, 0.5, a.mode, n_threads=threads, want_lut=False)
    t_cpu = time.perf_counter() - t
    with n5.open_file(data, 'r') as f:
        same = bool(np.array_equal(f['segmentation/cc0'][:], ref['labels']))
    nvox = int(np.prod(shape))
    best = min(runs, key=lambda r: r['workflow_wall_s'])
    line = {
        'workload': 'C1: ThresholdedComponentsWorkflow on a (125, 1250, 1250) float32 gzip N5 dataset '
                    '(synthetic CREMI-sized boundary map), block [50, 512, 512], threshold 0.5 %s, '
                    "target 'local', max_jobs 16" % a.mode,
        'voxels': nvox, 'runs': runs,
        'label_host_gvox_s': round(nvox / best['h2d_device_d2h_s'] / 1e9, 3),
        'job_gvox_s': round(nvox / sum(best[k] for k in ('n5_read_s', 'h2d_device_d2h_s', 'n5_write_s')) / 1e9, 3),
        'workflow_gvox_s': round(nvox / best['workflow_wall_s'] / 1e9, 3),
        'input_n5_write_s': round(t_in, 3),
        'labels_equal_oracle': same,
        'cpu_baseline': {'value': round(nvox / t_cpu / 1e9, 4), 'unit': 'Gvox/s', 'cores': threads, 'kind': 'port',
                         'sample': 'oracle/cc_oracle.c on the same volume in memory (no N5 / gzip), %.2f s' % t_cpu},
    }
    print(json.dumps(line), flush=True)
    if not a.out:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == '__main__':
    main()
