"""Timing of the stage-level entry points (one reference job each, run when a stage task is used on
its own: fused=False) on C3 (1024, 2048, 2048), block (64, 512, 512), 'greater' 0.5:
cc_block_components -> cc_merge_offsets -> cc_block_faces -> cc_merge_assignments -> cc_write
(block_components.py:236-291, merge_offsets.py:83-131, block_faces.py:87-177,
merge_assignments.py:88-141, write.py:185-220).  Prints one JSON line: per-kernel ms and achieved
GB/s at the algorithmic bytes (k_write_offsets 16 B/voxel: uint64 read + write in place;
k_face_pairs 16 B per face-voxel position: the two uint64 labels facing each other)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from cluster_tools_amd import _lib
    mode = sys.argv[1] if len(sys.argv) > 1 else 'greater'
    shape, bs, steps = (1024, 2048, 2048), (64, 512, 512), 5
    ctx = _lib.Context(0)
    x = ctx.generate_boundary_map(shape)
    local = torch.empty(shape, dtype=torch.int64, device=x.device)
    wall = {}

    def step(record):
        t = time.perf_counter()
        _, values = ctx.block_components(x, bs, 0.5, mode, out_dev=local)
        t1 = time.perf_counter()
        offsets, _, n_labels = _lib.merge_offsets(values)
        pairs = ctx.block_faces(local, bs, offsets)
        t2 = time.perf_counter()
        lut = ctx.merge_assignments(pairs, n_labels)
        t3 = time.perf_counter()
        ctx.write(local, bs, offsets, lut)
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        if record:
            for k, v in (('block_components', t1 - t), ('block_faces', t2 - t1), ('merge_assignments', t3 - t2),
                         ('write', t4 - t3)):
                wall[k] = wall.get(k, 0.0) + v / steps
        return len(pairs), n_labels

    for _ in range(2):
        step(False)
    ctx.reset_profile()
    ctx.set_profiling(1)
    for _ in range(steps):
        n_pairs, n_labels = step(True)
    prof = ctx.profile()
    ctx.set_profiling(0)
    k = {n: v['total_ms'] / steps for n, v in prof.items()}
    n = x.numel()
    face_vox = sum(((s - 1) // b) * (n // s) for s, b in zip(shape, bs))
    alg = {'k_write_offsets': 16.0 * n, 'k_face_pairs': 16.0 * face_vox}
    roof = {}
    for name, b in alg.items():
        if name in k:
            ach = b / (k[name] * 1e-3) / 1e9
            roof[name] = {'alg_bytes': int(b), 'ms': round(k[name], 4), 'achieved_gbs': round(ach, 1),
                          'frac': round(ach / 8000.0, 4)}
    print(json.dumps({'workload': 'C3 stage path (%s)' % mode, 'n_pairs': int(n_pairs), 'n_labels': int(n_labels),
                      'wall_ms_per_stage': {a: round(v * 1e3, 3) for a, v in wall.items()},
                      'roofline': roof,
                      'kernels_ms_per_step': {a: round(v, 4) for a, v in sorted(k.items(), key=lambda kv: -kv[1])}}))
    ctx.close()


if __name__ == '__main__':
    main()
