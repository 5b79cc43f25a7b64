"""Timing of the input-side kernels that have no bench of their own, on C3
(1024, 2048, 2048), block (64, 512, 512): the resized-mask map (cc_resize_mask_nearest, a
(512, 1024, 1024) mask to the volume's shape: k_mask_xmap + k_mask_resize, 0.5 + 4 B/voxel-ish)
and the 4-D watershed input (cc_normalize_channels over 3 float32 channels, agg mean:
k_block_stats per channel + k_norm_agg, 12 B read + 4 B written per voxel).  Prints one JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(f, reps=3):
    import torch
    f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    import torch
    from cluster_tools_amd import _lib
    shape, bs = (1024, 2048, 2048), (64, 512, 512)
    dev = torch.device('cuda', 0)
    ctx = _lib.Context(0)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    n = shape[0] * shape[1] * shape[2]
    small = (torch.rand((512, 1024, 1024), device=dev) > 0.5).to(torch.uint8)
    ms_mask = timed(lambda: ctx.resize_mask(small, shape))
    del small
    torch.cuda.empty_cache()
    x = ctx.generate_boundary_map(shape, device=dev)
    x4 = torch.empty((3,) + shape, dtype=torch.float32, device=dev)
    x4[0] = x
    x4[1] = x * 0.5
    x4[2] = 1.0 - x
    del x
    out = torch.empty(shape, dtype=torch.float32, device=dev)
    ms_norm = timed(lambda: ctx.normalize_channels(x4, bs, 'mean', out=out))
    print(json.dumps({'workload': 'C3 %s block %s' % (shape, bs),
                      'resize_mask_ms': round(ms_mask, 3), 'resize_mask_gbs_out': round(n / ms_mask / 1e6, 1),
                      'normalize_channels_3_mean_ms': round(ms_norm, 3),
                      'normalize_channels_gbs': round(n * 16 / ms_norm / 1e6, 1)}))
    ctx.close()


if __name__ == '__main__':
    main()
