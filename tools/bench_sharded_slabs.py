"""Multi-GPU readiness without a multi-GPU node: the z-slab schedule for N slabs
run one after another in ONE process on one GPU (distributed.label_slabs_single_process: every
collective becomes a device copy / list operation), so the per-slab cost -- kernels, host
synchronisations, launch gaps -- is measured without rank contention.  Workloads:
  c4  (1024, 2048, 2048) + ellipsoid mask, block (64, 512, 512), N slabs of 1024 / N planes
      (strong scaling: at N = 8 each rank would own a (128, 2048, 2048) slab)
  c3  the same without the mask
The single-volume step of the same volume (cc_label_volume) is timed beside it: the target is
per-slab time <= 1.15 x (single-volume step / N).  Prints one JSON line.
Usage: python tools/bench_sharded_slabs.py [N] [c4|c3] [steps] [sync]"""
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
    from cluster_tools_amd.synthetic import ellipsoid_mask_device
    a = sys.argv[1:]
    n = int(a[0]) if a else 8
    wl = a[1] if len(a) > 1 else 'c4'
    steps = int(a[2]) if len(a) > 2 else 5
    sched = a[3] if len(a) > 3 else None        # 'sync': the host-synchronised schedule (evidence of its kernels)
    shape, bs = (1024, 2048, 2048), (64, 512, 512)
    dev = torch.device('cuda', 0)
    ctxs = [_lib.Context(0) for _ in range(n)]
    for c in ctxs:
        c.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    x = ctxs[0].generate_boundary_map(shape, device=dev)
    mask = ellipsoid_mask_device(shape, 0, shape[0], dev) if wl == 'c4' else None
    torch.cuda.synchronize()
    # single-volume step of the same volume (the denominator)
    out = torch.empty(shape, dtype=torch.int64, device=dev)
    for _ in range(2):
        ctxs[0].label_volume(x, bs, 0.5, 'greater', mask=mask, out=out)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        ctxs[0].label_volume(x, bs, 0.5, 'greater', mask=mask, out=out)
    torch.cuda.synchronize()
    single_ms = (time.perf_counter() - t0) / steps * 1e3
    del out
    torch.cuda.empty_cache()
    for _ in range(2):
        label_slabs_single_process(ctxs, x, bs, 0.5, 'greater', mask=mask, schedule=sched)
    torch.cuda.synchronize()
    ctxs[0].reset_profile()                  # host_* counters are library-wide
    t0 = time.perf_counter()
    for _ in range(steps):
        o, res, sums, luts = label_slabs_single_process(ctxs, x, bs, 0.5, 'greater', mask=mask, schedule=sched)
        del o
    torch.cuda.synchronize()
    slabs_ms = (time.perf_counter() - t0) / steps * 1e3
    host = {k: {'count': v['count'] / steps / n, 'ms': round(v['total_ms'] / steps / n, 4)}
            for k, v in ctxs[0].profile().items() if k.startswith('host_')}
    # per-kernel times of one slab step (every launch timed, untimed pass)
    for c in ctxs:
        c.set_profiling(1)
        c.reset_profile()
    o, res, sums, luts = label_slabs_single_process(ctxs, x, bs, 0.5, 'greater', mask=mask, schedule=sched)
    torch.cuda.synchronize()
    per = []
    for c in ctxs:
        p = c.profile()
        per.append({k: round(v['total_ms'], 4) for k, v in sorted(p.items(), key=lambda kv: -kv[1]['total_ms'])
                    if v['count'] and not k.startswith('host_')})
        c.set_profiling(0)
    mid = per[n // 2]
    print(json.dumps({
        'workload': '%s %s block %s as %d z-slabs in one process' % (wl, shape, bs, n),
        'schedule': sched or 'default',
        'single_volume_step_ms': round(single_ms, 3), 'all_slabs_ms': round(slabs_ms, 3),
        'per_slab_ms': round(slabs_ms / n, 3), 'target_per_slab_ms': round(1.15 * single_ms / n, 3),
        'ratio_to_ideal': round(slabs_ms / single_ms, 4),
        'host_per_slab': host,
        'middle_slab_kernels_ms': mid, 'middle_slab_kernel_sum_ms': round(sum(mid.values()), 4),
        'seam_forms': sorted(set(r.get('seam_form', '') for r in res)) if res else []}))
    for c in ctxs:
        c.close()


if __name__ == '__main__':
    main()
