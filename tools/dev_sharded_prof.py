"""dev: per-kernel times of the z-slab (multi-GPU) schedule without rank contention: several
slabs on ONE GPU in one process (distributed.label_slabs_single_process), each slab its own
context with HIP-event profiling; prints one JSON line per slab.
Usage: python tools/dev_sharded_prof.py [n_slabs] [slab_z] [Y] [X] [mode]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from cluster_tools_amd import _lib
    from cluster_tools_amd.distributed import label_slabs_single_process
    a = sys.argv[1:]
    n, zs, Y, X = (int(v) for v in (a + ['2', '256', '4096', '4096'][len(a):])[:4])
    mode = a[4] if len(a) > 4 else 'greater'
    dev = torch.device('cuda', 0)
    ctxs = [_lib.Context(0) for _ in range(n)]
    x = ctxs[0].generate_boundary_map((n * zs, Y, X), origin=(0, 0, 0), device=dev)
    bs = (64, 512, 512)
    for c in ctxs:
        c.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    label_slabs_single_process(ctxs, x, bs, 0.5, mode)          # warm-up
    for c in ctxs:
        c.set_profiling(1)
        c.reset_profile()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out, res, sums, luts = label_slabs_single_process(ctxs, x, bs, 0.5, mode)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    for i, c in enumerate(ctxs):
        p = c.profile()
        print(json.dumps({'slab': i, 'total_ms_all_slabs': round(dt * 1e3, 3),
                          'kernels_ms': {k: round(v['total_ms'], 4) for k, v in
                                         sorted(p.items(), key=lambda kv: -kv[1]['total_ms']) if v['count']},
                          'result': res[i]}))


if __name__ == '__main__':
    main()
