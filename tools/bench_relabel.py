"""Timing of the device consecutive relabel (cc_relabel_consecutive, reference RelabelWorkflow)
on the C3 'less' labels (150 k ids).  Prints one JSON line: Gvox/s, the end-to-end fraction of
8 TB/s at 24 B/voxel (the id set pass reads 8 B, the apply pass reads 8 B and writes 8 B) and the
roofline of each of the two volume kernels."""
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
    lab, _ = ctx.label_volume(x, bs, 0.5, 'less')
    del x
    out = torch.empty_like(lab)
    for _ in range(2):
        ctx.relabel_consecutive(lab, out=out)
    t0 = time.perf_counter()
    for _ in range(steps):
        ctx.relabel_consecutive(lab, out=out)
    dt = (time.perf_counter() - t0) / steps
    ctx.reset_profile()
    ctx.set_profiling(1)
    for _ in range(steps):
        ctx.relabel_consecutive(lab, out=out)
    prof = ctx.profile()
    ctx.set_profiling(0)
    k = {n: v['total_ms'] / steps for n, v in prof.items()}
    n = lab.numel()
    roof = {}
    for name, bpv in (('k_rl_apply', 16.0), ('k_rl_unique', 8.0)):     # 8 B read (+ 8 B write)
        ach = n * bpv / (k[name] * 1e-3) / 1e9
        roof[name] = {'bound': 'hbm', 'achieved': round(ach, 1), 'peak': 8000.0, 'unit': 'GB/s',
                      'frac': round(ach / 8000.0, 4), 'alg_bytes_per_voxel': bpv}
    print(json.dumps({'metric': 'Gvoxels/sec consecutive relabel end-to-end', 'value': round(n / dt / 1e9, 3),
                      'unit': 'Gvox/s', 'ms_per_step': round(dt * 1e3, 3),
                      'e2e_frac': round(n * 24.0 / dt / 1e9 / 8000.0, 4), 'roofline': roof,
                      'kernels_ms_per_step': {n: round(v, 4) for n, v in sorted(k.items(), key=lambda kv: -kv[1])}}))
    ctx.close()


if __name__ == '__main__':
    main()
