"""Worker of tests/test_gpu_sharded.py::test_two_ranks_one_gpu_gloo (launched by torch.distributed.run):
one rank of the z-slab schedule with a real libcc_mi355x context on cuda:0, collectives over gloo
staged through host memory (distributed.StagedComm), or -- one rank, argv[5] == 'nccl' -- over
RCCL on GPU tensors (distributed.TorchComm, the production communicator)."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out_dir, mode = sys.argv[1], sys.argv[2]
    shape = tuple(int(v) for v in sys.argv[3].split(','))
    block_shape = tuple(int(v) for v in sys.argv[4].split(','))
    backend = sys.argv[5] if len(sys.argv) > 5 else 'gloo'
    dev = torch.device('cuda', 0)
    if backend == 'nccl':                    # RCCL: one rank per GPU, collectives on GPU tensors
        torch.cuda.set_device(dev)
        dist.init_process_group('nccl', device_id=dev)
    else:
        dist.init_process_group('gloo')
    rank, world = dist.get_rank(), dist.get_world_size()
    from cluster_tools_amd import _lib
    from cluster_tools_amd.distributed import ShardedLabeler, StagedComm, TorchComm, slab_bounds
    from oracle import oracle as O
    z0, zs = slab_bounds(shape[0], block_shape[0], world)[rank]
    x = torch.from_numpy(O.boundary_map((zs,) + shape[1:], origin=(z0, 0, 0), n_threads=1)).to(dev)
    with _lib.Context(0) as ctx:
        ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        lab = ShardedLabeler(ctx, shape, block_shape, z0, zs, dev, comm=TorchComm(device=dev) if backend == 'nccl' else StagedComm(device=dev))
        lab.label(x, 0.5, mode)                # twice more below: workspace reuse across runs
        out = torch.empty(tuple(x.shape), dtype=torch.int64, device=dev)
        res = lab.label(x, 0.5, mode, out=out)
        torch.cuda.synchronize()
    np.save(os.path.join(out_dir, 'slab_%d.npy' % rank), out.cpu().numpy())
    np.save(os.path.join(out_dir, 'nl_%d.npy' % rank), np.array([res['n_labels']], dtype=np.int64))
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
