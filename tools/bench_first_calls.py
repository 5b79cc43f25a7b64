"""First-call cost of the secondary device tasks in a fresh process (relabel's
first k_rl_unique took 666 ms and evaluation's first k_ev_overlaps 80 ms while their hash tables
grew): C3 'greater' / 'less' labels (150 k ids), then cc_relabel_consecutive and cc_evaluate,
each timed on the first and the second call.  Prints one JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from cluster_tools_amd import _lib
    shape, bs = (1024, 2048, 2048), (64, 512, 512)
    ctx = _lib.Context(0)
    x = ctx.generate_boundary_map(shape)
    seg, _ = ctx.label_volume(x, bs, 0.5, 'greater')
    gt, r = ctx.label_volume(x, bs, 0.5, 'less')
    del x
    torch.cuda.synchronize()
    out = {'workload': 'C3 labels: seg = greater, gt = less (%d ids)' % r['n_labels']}
    tmp = torch.empty_like(gt)
    for k in ('relabel_first_ms', 'relabel_second_ms'):
        t0 = time.perf_counter()
        ctx.relabel_consecutive(gt, out=tmp)
        torch.cuda.synchronize()
        out[k] = round((time.perf_counter() - t0) * 1e3, 3)
    for k in ('evaluate_first_ms', 'evaluate_second_ms'):
        ctx.reset_profile()
        ctx.set_profiling(1)
        t0 = time.perf_counter()
        res = ctx.evaluate(seg, gt, bs)
        torch.cuda.synchronize()
        out[k] = round((time.perf_counter() - t0) * 1e3, 3)
        ctx.set_profiling(0)
        out[k.replace('_ms', '_kernels')] = {a: round(v['total_ms'], 3) for a, v in ctx.profile().items()}
    out['n_pairs'] = res['n_pairs']
    print(json.dumps(out))
    ctx.close()


if __name__ == '__main__':
    main()
