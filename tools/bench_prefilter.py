"""Timing of the input-preparation kernels on C3-sized volumes: cc_channel_mean (3 float32
channels -> float32 mean: 16 B/voxel algorithmic) and cc_gaussian_smooth_blocks (sigma_prefilter:
k_block_stats 4 B/voxel, then the z / y / x passes 8 B/voxel each).  Prints one JSON line with the
per-kernel times and their HBM rooflines.

    python tools/bench_prefilter.py [--steps 5] [--sigma 1.0] [--shape Z,Y,X]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--steps', type=int, default=5)
    p.add_argument('--sigma', type=float, default=1.0)
    p.add_argument('--shape', default='1024,2048,2048')
    a = p.parse_args()
    import torch
    from cluster_tools_amd import _lib
    shape = tuple(int(v) for v in a.shape.split(','))
    bs = (64, 512, 512)
    ctx = _lib.Context(0)
    dev = torch.device('cuda', 0)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    n = 1
    for s in shape:
        n *= s
    x = ctx.generate_boundary_map(shape, dither=True)
    stack = torch.empty((3,) + shape, dtype=torch.float32, device=dev)
    for c in range(3):
        stack[c].copy_(x)
    out = torch.empty(shape, dtype=torch.float32, device=dev)
    res = {}

    def timed(name, fn):
        fn()
        torch.cuda.synchronize()
        ctx.reset_profile()
        ctx.set_profiling(1)
        t0 = time.perf_counter()
        for _ in range(a.steps):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        prof = ctx.profile()
        ctx.set_profiling(0)
        res[name] = {'ms_per_call': round(dt * 1e3, 3),
                     'kernels_ms': {k: round(v['total_ms'] / a.steps, 4) for k, v in prof.items() if v['count']}}

    timed('channel_mean', lambda: ctx.channel_mean(stack, [0, 1, 2], out=out))
    del stack
    torch.cuda.empty_cache()
    timed('gaussian', lambda: ctx.gaussian_smooth_blocks(x, bs, a.sigma, out=out))
    roof = {}
    for call, kern, b in (('channel_mean', 'k_channel_mean', 16.0), ('gaussian', 'k_block_stats', 4.0),
                          ('gaussian', 'k_gauss_z', 8.0), ('gaussian', 'k_gauss_y', 8.0), ('gaussian', 'k_gauss_x', 8.0)):
        ms = res[call]['kernels_ms'].get(kern)
        if ms:
            ach = n * b / (ms * 1e-3) / 1e9
            roof[kern] = {'ms': ms, 'alg_bytes_per_voxel': b, 'achieved_gbs': round(ach, 1),
                          'frac': round(ach / 8000.0, 4)}
    print(json.dumps({'shape': list(shape), 'block_shape': list(bs), 'sigma': a.sigma,
                      'gvox_per_s': {k: round(n / (v['ms_per_call'] * 1e-3) / 1e9, 2) for k, v in res.items()},
                      'calls': res, 'roofline': roof}))
    ctx.close()


if __name__ == '__main__':
    main()
