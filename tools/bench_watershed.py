"""Timing of the device seeded watershed (cc_watershed_from_seeds, WatershedFromSeeds of
ThresholdAndWatershedWorkflow) on C3 (1024, 2048, 2048), block (64, 512, 512): seeds = the
'less' components of the synthetic boundary map (cell interiors), input = the map.  Prints one
JSON line: ms per call, relaxation rounds, per-kernel ms."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from cluster_tools_amd import _lib
    shape = tuple(int(v) for v in (sys.argv[1].split(',') if len(sys.argv) > 1 else (1024, 2048, 2048)))
    bs = (64, 512, 512)
    ctx = _lib.Context(0)
    x = ctx.generate_boundary_map(shape)
    seeds, res = ctx.label_volume(x, bs, 0.5, 'less')
    out = torch.empty_like(seeds)
    ctx.watershed_from_seeds(x, seeds, bs, out=out)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    _, rounds = ctx.watershed_from_seeds(x, seeds, bs, out=out)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ctx.reset_profile()
    ctx.set_profiling(1)
    ctx.watershed_from_seeds(x, seeds, bs, out=out)
    prof = ctx.profile()
    ctx.set_profiling(0)
    n = x.numel()
    unl = int((out == 0).sum().item())
    print(json.dumps({'workload': 'C3 %s block %s, seeds = CCL less (%d components)' % (shape, bs, res['n_components']),
                      'ms': round(dt * 1e3, 3), 'gvox_s': round(n / dt / 1e9, 3), 'rounds': rounds,
                      'unlabelled_voxels': unl,
                      'kernels_ms': {k: round(v['total_ms'], 3) for k, v in
                                     sorted(prof.items(), key=lambda kv: -kv[1]['total_ms'])}}))
    ctx.close()


if __name__ == '__main__':
    main()
