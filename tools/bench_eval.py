"""Timing of the device evaluation (cc_evaluate, reference EvaluationWorkflow) on the C3 volume.

    python tools/bench_eval.py [--shape Z,Y,X] [--steps K] [--warmup W]

seg = the CCL labels at 'greater 0.5', gt = the CCL labels at 'less 0.5' of the same synthetic
boundary map (both uint64, resident in HBM).  One step = one cc_evaluate call (overlaps, fold,
sizes, reductions, host measures).  Prints one JSON line: Gvox/s end to end and the roofline of
k_ev_overlaps at 16 algorithmic bytes per voxel (seg + gt uint64 reads), from HIP events.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

HBM_PEAK_GBS = 8000.0


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--shape', default='1024,2048,2048')
    p.add_argument('--block-shape', default='64,512,512')
    p.add_argument('--steps', type=int, default=10)
    p.add_argument('--warmup', type=int, default=2)
    a = p.parse_args()
    import torch
    from cluster_tools_amd import _lib
    shape = tuple(int(v) for v in a.shape.split(','))
    bs = tuple(int(v) for v in a.block_shape.split(','))
    ctx = _lib.Context(0)
    inp = ctx.generate_boundary_map(shape)
    seg, _ = ctx.label_volume(inp, bs, 0.5, 'greater')
    gt, _ = ctx.label_volume(inp, bs, 0.5, 'less')
    del inp
    torch.cuda.synchronize()
    for _ in range(a.warmup):
        ctx.evaluate(seg, gt, bs)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        res = ctx.evaluate(seg, gt, bs)
    dt = (time.perf_counter() - t0) / a.steps
    ctx.reset_profile()
    ctx.set_profiling(1)
    for _ in range(a.steps):
        ctx.evaluate(seg, gt, bs)
    prof = ctx.profile()
    ctx.set_profiling(0)
    nvox = seg.numel()
    k = prof['k_ev_overlaps']
    kms = k['total_ms'] / k['count']
    achieved = nvox * 16.0 / (kms * 1e-3) / 1e9
    print(json.dumps({
        'metric': 'Gvoxels/sec segmentation evaluation (overlaps + VI / rand) end-to-end',
        'value': round(nvox / dt / 1e9, 3), 'unit': 'Gvox/s', 'ms_per_step': round(dt * 1e3, 3),
        'steps': a.steps, 'config': {'shape': shape, 'block_shape': bs, 'seg': 'CCL greater 0.5',
                                      'gt': 'CCL less 0.5', 'ignore_label': 0},
        'roofline': {'bound': 'hbm', 'kernel': 'k_ev_overlaps', 'achieved': round(achieved, 1),
                     'peak': HBM_PEAK_GBS, 'unit': 'GB/s', 'frac': round(achieved / HBM_PEAK_GBS, 4),
                     'alg_bytes_per_voxel': 16.0, 'avg_launch_ms': round(kms, 4)},
        'kernels_ms_per_step': {n: round(v['total_ms'] / a.steps, 4) for n, v in
                                sorted(prof.items(), key=lambda kv: -kv[1]['total_ms'])},
        'result': res}))
    ctx.close()


if __name__ == '__main__':
    main()
