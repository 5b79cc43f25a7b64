"""Timing of the device Threshold task (cc_threshold: by default k_sample/k_guess -> k_thr_spec -> k_params_verify
-> k_thr_fix of the listed tiles; CC_THRESHOLD_TWO_PASS=1 selects k_block_stats + k_block_params + k_threshold,
reference thresholded_components/threshold.py) on C3.  Prints one JSON line: Gvox/s and the
roofline of the two volume kernels at their algorithmic bytes (k_block_stats 4 B/voxel read,
k_threshold 4 B read + 1 B uint8 write)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from cluster_tools_amd import _lib
    shape, bs, steps = (1024, 2048, 2048), (64, 512, 512), 10
    ctx = _lib.Context(0)
    x = ctx.generate_boundary_map(shape)
    out = torch.empty(shape, dtype=torch.uint8, device=x.device)
    for _ in range(2):
        ctx.threshold(x, bs, 0.5, 'greater', out=out)
    t0 = time.perf_counter()
    for _ in range(steps):
        ctx.threshold(x, bs, 0.5, 'greater', out=out)
    dt = (time.perf_counter() - t0) / steps
    ctx.reset_profile()
    ctx.set_profiling(1)
    for _ in range(steps):
        ctx.threshold(x, bs, 0.5, 'greater', out=out)
    prof = ctx.profile()
    ctx.set_profiling(0)
    k = {n: v['total_ms'] / steps for n, v in prof.items()}
    n = x.numel()
    roof = {}
    for name, b in (('k_block_stats', 4.0), ('k_threshold', 5.0), ('k_thr_spec', 5.0)):
        if name in k:
            ach = n * b / (k[name] * 1e-3) / 1e9
            roof[name] = {'achieved_gbs': round(ach, 1), 'frac': round(ach / 8000.0, 4), 'alg_bytes_per_voxel': b}
    print(json.dumps({'metric': 'Gvoxels/sec Threshold task (normalize + threshold -> uint8)',
                      'variant': 'two_pass' if os.environ.get('CC_THRESHOLD_TWO_PASS') == '1' else 'speculative',
                      'e2e_frac_at_5B': round(n * 5.0 / dt / 1e9 / 8000.0, 4),
                      'value': round(n / dt / 1e9, 3), 'unit': 'Gvox/s', 'ms_per_step': round(dt * 1e3, 3),
                      'roofline': roof,
                      'kernels_ms_per_step': {a: round(v, 4) for a, v in sorted(k.items(), key=lambda kv: -kv[1])}}))
    ctx.close()


if __name__ == '__main__':
    main()
