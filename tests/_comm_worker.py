"""Worker of tests/test_gpu_comm_ranks.py: ONE rank of the library's own sharded C entry
(cc_comm_create / cc_label_volume_sharded) on cuda:0, with the collectives served by the
test-only RCCL stand-in (tests/fake_rccl, loaded through CC_RCCL_PATH by the parent) so that 2-8
ranks can share the one GPU of a test box.

argv[1]: JSON spec {out, rank, world, uid (hex), shape, origin, mode, mask, generate (the slab made
on the device by cc_generate_boundary_map), hash_only (an xxh64 digest of the labels instead of
the array), calls: [...]}; each
call: {block_shape, z_shift (this rank's z_offset moved by this much: a bad slab), src ('host' |
'kernel' | 'kernel_side': the slab written by a torch kernel queued behind a GPU sleep, on the
default or a side stream, with no synchronisation before the call)}.
Writes out/rank<r>.json (per call: ok / error text, seconds, result, cc_comm_info) and the
slab labels of each successful call as out/rank<r>_call<k>.npy."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    spec = json.loads(sys.argv[1])
    import torch
    from cluster_tools_amd import _lib
    from cluster_tools_amd.distributed import slab_bounds
    from oracle import oracle as O
    rank, world = spec['rank'], spec['world']
    shape, origin = tuple(spec['shape']), tuple(spec['origin'])
    dev = torch.device('cuda', 0)
    log = {'calls': []}
    with _lib.Context(0) as ctx, _lib.Comm(bytes.fromhex(spec['uid']), world, rank, 0) as comm:
        for k, call in enumerate(spec['calls']):
            bs = tuple(call['block_shape'])
            z0, zs = slab_bounds(shape[0], bs[0], world)[rank]
            if spec.get('generate'):          # full-size runs: the slab made on the device
                x = ctx.generate_boundary_map((zs,) + shape[1:], origin=(origin[0] + z0,) + origin[1:])
            else:
                x = O.boundary_map((zs,) + shape[1:], origin=(origin[0] + z0,) + origin[1:], n_threads=1)
            m = None
            if spec.get('mask') and spec.get('generate'):
                from cluster_tools_amd.synthetic import ellipsoid_mask_device
                m = ellipsoid_mask_device(shape, z0, zs, dev)
            elif spec.get('mask'):
                from oracle.synth import ellipsoid_mask
                m = torch.from_numpy(np.ascontiguousarray(ellipsoid_mask(shape)[z0:z0 + zs])).to(dev)
            src = call.get('src', 'host')
            xh = x if spec.get('generate') else torch.from_numpy(x).to(dev)
            torch.cuda.synchronize()
            side = torch.cuda.Stream(dev) if src == 'kernel_side' else None
            with torch.cuda.stream(side) if side is not None else torch.cuda.stream(torch.cuda.default_stream(dev)):
                if src.startswith('kernel'):
                    # the slab is written by a kernel that starts only after ~50 ms of GPU sleep on
                    # the current stream; the call must be ordered after it
                    xd = torch.empty_like(xh)
                    xd.fill_(float('nan'))
                    torch.cuda._sleep(120_000_000)
                    torch.mul(xh, 1.0, out=xd)
                else:
                    xd = xh
                t0 = time.time()
                try:
                    lab, res = ctx.label_volume_sharded(comm, xd, shape, z0 + call.get('z_shift', 0), bs, 0.5,
                                                        spec['mode'], mask=m)
                    torch.cuda.current_stream(dev).synchronize()
                    entry = {'ok': True, 'res': res, 'label_seconds': time.time() - t0}
                    if spec.get('hash_only'):     # full-size runs: a digest of the slab's labels
                        import xxhash
                        entry['xxh64'] = xxhash.xxh64(lab.cpu().numpy().data).hexdigest()
                    else:
                        np.save(os.path.join(spec['out'], 'rank%d_call%d.npy' % (rank, k)), lab.cpu().numpy())
                except RuntimeError as e:
                    entry = {'ok': False, 'error': str(e)}
                entry['seconds'] = time.time() - t0
                entry['info'] = comm.info()
                entry['z0'], entry['zs'] = z0, zs
                log['calls'].append(entry)
    with open(os.path.join(spec['out'], 'rank%d.json' % rank), 'w') as f:
        json.dump(log, f)


if __name__ == '__main__':
    main()
