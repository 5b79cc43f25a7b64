"""Cold start of a one-shot drop-in job on BASELINE config 1's geometry (125, 1250, 1250), block
(50, 512, 512), 'greater' 0.5: every target='local' job is a fresh process making ONE library call,
so its first-call costs are what the job pays.  In a fresh process:
ctx creation, the input upload, then the FIRST cc_label_volume (cold) and the next ones (warm),
each bracketed by device synchronisation.  The library's per-launch HIP events and its host-side
allocation accounting ("host_alloc": hipMalloc calls and time) break the first call down.
Prints one JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    t_imp = time.perf_counter()
    import numpy as np
    import torch
    from cluster_tools_amd import _lib
    from oracle import oracle as O
    shape, bs = (125, 1250, 1250), (50, 512, 512)
    host = O.boundary_map(shape, n_threads=16)             # host input, as read from N5
    torch.cuda.init()
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    x = torch.from_numpy(host).to(dev)
    out = torch.empty(shape, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ctx = _lib.Context(0)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    t_create = time.perf_counter() - t0
    ctx.set_profiling(1)
    ctx.reset_profile()
    t0 = time.perf_counter()
    _, res = ctx.label_volume(x, bs, 0.5, 'greater', out=out)
    torch.cuda.synchronize()
    cold = time.perf_counter() - t0
    cold_prof = ctx.profile()
    ctx.set_profiling(0)
    warm = []
    for _ in range(5):
        t0 = time.perf_counter()
        ctx.label_volume(x, bs, 0.5, 'greater', out=out)
        torch.cuda.synchronize()
        warm.append(time.perf_counter() - t0)
    kern_ms = sum(v['total_ms'] for k, v in cold_prof.items() if not k.startswith('host_'))
    print(json.dumps({
        'workload': 'C1 geometry %s block %s (one-shot drop-in job)' % (shape, bs),
        'ctx_create_ms': round(t_create * 1e3, 3), 'cold_call_ms': round(cold * 1e3, 3),
        'warm_call_ms': round(min(warm) * 1e3, 3), 'warm_calls_ms': [round(w * 1e3, 3) for w in warm],
        'cold_kernel_event_ms': round(kern_ms, 3),
        'cold_host_alloc': cold_prof.get('host_alloc'), 'cold_host_sync': cold_prof.get('host_sync'),
        'cold_breakdown_ms': {k: round(v['total_ms'], 3) for k, v in
                              sorted(cold_prof.items(), key=lambda kv: -kv[1]['total_ms'])},
        'n_labels': res['n_labels'], 'process_s_to_first_call': round(time.perf_counter() - t_imp, 2)}))
    ctx.close()


if __name__ == '__main__':
    main()
