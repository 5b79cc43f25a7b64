"""One rank of a z-slab sharded BlockComponents job (config 'gpus' > 1).

Started by block_components._fused_sharded as
    python -m torch.distributed.run --nproc-per-node N ... sharded_job.py <job config> <out dir>
Rank r owns the z-slab slab_bounds(Z, block_shape[0], N)[r] (block faces at slab seams, so every
per-block stage stays local).  It reads its slab from the input N5 dataset (and mask), labels it
with distributed.ShardedLabeler (RCCL: allgather of slab sums, one plane to rank r + 1, padded
allgather of the seam pairs, replicated union-find), writes its slab of the final labels to the
output N5 dataset and saves its block values / LUT part / timings to <out dir>/rank_<r>.npz for
the job process to assemble.  Reference counterpart: the ProcessPool of block jobs
(cluster_tools/cluster_tasks.py:301-335, 545-551), with file hand-offs between stages.
"""
import json
import os
import sys
import time

import numpy as np


def main(config_path, out_dir):
    import torch
    import torch.distributed as dist
    from cluster_tools_amd import _lib
    from cluster_tools_amd.distributed import ShardedLabeler, StagedComm, slab_bounds
    from cluster_tools_amd.thresholded_components import block_components as bc
    import cluster_tools_amd.utils.volume_utils as vu

    with open(config_path) as f:
        config = json.load(f)
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    local_rank = int(os.environ.get('LOCAL_RANK', rank))
    backend = config.get('dist_backend', 'nccl')
    from cluster_tools_amd.distributed import check_rccl_ranks
    check_rccl_ranks(backend, local_rank, int(os.environ.get('LOCAL_WORLD_SIZE', world)))
    gpu = local_rank if backend == 'nccl' else local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(gpu)
    dev = torch.device('cuda', gpu)
    if backend == 'nccl':
        dist.init_process_group('nccl', device_id=dev)
    else:
        dist.init_process_group(backend)

    shape = tuple(vu.get_shape(config['input_path'], config['input_key']))
    if config.get('channel') is not None:
        shape = shape[1:]            # 4-D (C, Z, Y, X) input, channels averaged on the device
    bs = tuple(config['block_shape'])
    bounds = slab_bounds(shape[0], bs[0], world)
    z0, zs = bounds[rank]
    box = [(z0, z0 + zs), (0, shape[1]), (0, shape[2])]
    threads = max(1, bc._n_threads() // world)
    timing = {}

    t = time.perf_counter()
    inp, chans = bc.read_input(config, box)
    mask, resized = bc.read_mask(config, shape, box)
    timing['n5_read_s'] = time.perf_counter() - t
    ctx = _lib.Context(gpu)
    t = time.perf_counter()
    x = torch.from_numpy(inp if chans is None else inp.reshape(-1).view(np.uint8)).to(dev)
    m = bc.device_mask(ctx, mask, resized, shape, dev, z0, zs)
    torch.cuda.synchronize(dev)
    timing['h2d_s'] = time.perf_counter() - t
    stack_shape, stack_dtype = inp.shape, inp.dtype
    del inp, mask

    if chans is not None or float(config.get('sigma_prefilter', 0) or 0) > 0:
        # input preparation (channel mean, sigma_prefilter: block-local, so slab-local)
        ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        t = time.perf_counter()
        if chans is not None:
            x = ctx.channel_mean(x, chans, shape4=stack_shape, dtype=stack_dtype)
        x = bc.prefilter(ctx, x, config)
        torch.cuda.synchronize(dev)
        timing['prefilter_s'] = time.perf_counter() - t
    comm = StagedComm(device=dev) if backend != 'nccl' else None
    lab = ShardedLabeler(ctx, shape, bs, z0, zs, dev, comm=comm)
    out = torch.empty(tuple(x.shape), dtype=torch.int64, device=dev)
    dist.barrier()
    t = time.perf_counter()
    res = lab.label(x, config['threshold'], config['threshold_mode'], mask=m, out=out)
    torch.cuda.synchronize(dev)
    timing['device_s'] = time.perf_counter() - t
    nby, nbx = -(-shape[1] // bs[1]), -(-shape[2] // bs[2])
    nb_slab = -(-zs // bs[0]) * nby * nbx
    values = ctx.block_values(nb_slab)
    lut_part = ctx.lut_local()
    del x, m
    t = time.perf_counter()
    labels = out.cpu().numpy().view(np.uint64)
    timing['d2h_s'] = time.perf_counter() - t
    del out

    # output slabs: chunk-aligned seams -> every rank writes its own chunks at once; otherwise a
    # chunk straddles two slabs and the ranks write one after another (read-merge-write)
    with vu.file_reader(config['output_path'], 'r') as f:
        cz = f[config['output_key']].chunks[0]
    aligned = all(b[0] % cz == 0 for b in bounds)
    t = time.perf_counter()
    if aligned:
        bc._write_output(config, labels, box, threads)
    else:
        for r in range(world):
            if r == rank:
                bc._write_output(config, labels, box, bc._n_threads())
            dist.barrier()
    timing['n5_write_s'] = time.perf_counter() - t
    ctx.close()
    np.savez(os.path.join(out_dir, 'rank_%i.npz' % rank), values=values, lut=lut_part,
             sum=np.uint64(lab.sums[rank]), n_components=np.uint64(res['n_components']),
             z0=z0, zs=zs, seam_form=res['seam_form'], **{k: np.float64(v) for k, v in timing.items()})
    dist.barrier()
    dist.destroy_process_group()


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
