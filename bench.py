"""Benchmark: Gvoxels/s of thresholded CCL end to end on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--mode greater|less] [--mask]

One step = the full five-stage path (block_components -> merge_offsets -> block_faces ->
merge_assignments -> write) over one synthetic volume that is already resident in HBM,
ending with the final uint64 labels resident in HBM.

Workloads (--workload).  One workload keeps its meaning at every N, so a
1 -> 2 -> 4 -> 8 series is one curve:
  c3 (default, every N)  (1024, 2048, 2048) float32, block (64, 512, 512), threshold 0.5 'greater';
       strong scaling: the one volume split into N z-slabs (N = 1: the headline single-GPU case)
  c4   C3 + the ellipsoid uint8 mask, strong-scaled the same way (BASELINE config 4)
  c5   weak scaling: each rank owns a (256, 4096, 4096) slab of a (256 N, 4096, 4096) volume --
       N = 1 is one such slab, N = 8 is C5, (2048, 4096, 4096)
  c2   (512, 512, 512), block (128, 128, 128)
  c1   (125, 1250, 1250), block (50, 512, 512): BASELINE config 1's geometry; the line also carries
       `cold_start`: a fresh process (a child of this one, input handed over as a .npy file) timing
       its FIRST cc_label_volume -- what every one-shot target='local' job pays -- and the warm calls
  --dither: continuous input (the map plus a sub-2^-8 dither).  N > 1 runs one process per GPU;
  seams are stitched over RCCL (cluster_tools_amd/distributed.py).

Launch: `python bench.py --gpus N` starts its own N ranks when it is not already one of them
(WORLD_SIZE unset): a child `python -m torch.distributed.run --nproc-per-node N bench.py ...` is
started BEFORE this process imports torch or loads the library (a subprocess, never an exec), its
stdout (rank 0's JSON line) is relayed, and the exit code is non-zero if any rank failed -- the
analogue of the reference's LocalTask pool (cluster_tools/cluster_tasks.py:545-551).  Under
`torch.distributed.run` (WORLD_SIZE set) this process is one rank.
Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = 'Gvoxels/sec thresholded CCL end-to-end at 1/2/4/8 MI355X; % of HBM roofline'
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
B_ALG = 12.0                   # algorithmic bytes / voxel: f32 read + uint64 write (+1 with mask)


def live_voxels(mask, block_shape):
    """Voxels of the blocks that hold a mask voxel: the only blocks whose input the reference reads
    (block_components.py:197-201 returns before reading the input of a block with an empty mask),
    so a masked run's algorithmic bytes are 8 + 1 per voxel + 4 per voxel of these blocks."""
    n = 0
    Z, Y, X = mask.shape
    for z in range(0, Z, block_shape[0]):
        for y in range(0, Y, block_shape[1]):
            for x in range(0, X, block_shape[2]):
                b = mask[z:z + block_shape[0], y:y + block_shape[1], x:x + block_shape[2]]
                if bool(b.any()):
                    n += b.numel()
    return n
# algorithmic bytes per voxel of each kernel
KERNEL_BYTES = {'k_spec': 4.0, 'k_pass2': 8.0}


WORKLOADS = {
    'c3': {'shape': (1024, 2048, 2048), 'block': (64, 512, 512), 'scaling': 'strong'},
    'c4': {'shape': (1024, 2048, 2048), 'block': (64, 512, 512), 'scaling': 'strong', 'mask': True},
    'c5': {'per_rank': (256, 4096, 4096), 'block': (64, 512, 512), 'scaling': 'weak'},
    'c2': {'shape': (512, 512, 512), 'block': (128, 128, 128), 'scaling': 'strong'},
    'c1': {'shape': (125, 1250, 1250), 'block': (50, 512, 512), 'scaling': 'strong'},
}


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--timed-prof', type=int, default=2,
                   help='HIP-event level inside the timed region: 2 volume kernels only, 1 every launch')
    p.add_argument('--steps', type=int, default=10)
    p.add_argument('--warmup', type=int, default=3)
    p.add_argument('--mode', default='greater')
    p.add_argument('--threshold', type=float, default=0.5)
    p.add_argument('--mask', action='store_true')
    p.add_argument('--dither', action='store_true',
                   help='continuous input: the synthetic map plus a deterministic sub-2^-8 dither (not quantized)')
    p.add_argument('--shape', default=None, help='override Z,Y,X (per-rank slab for N > 1)')
    p.add_argument('--workload', default='c3', choices=sorted(WORKLOADS),
                   help='c3 (default; strong-scaled z-slabs at N>1), c4 (C3 + mask, strong-scaled z-slabs), '
                        'c5 ((256N,4096,4096), weak), c2 (512^3, block 128^3), c1 (125x1250x1250, block '
                        '50x512x512, + cold_start)')
    p.add_argument('--block-shape', default=None)
    p.add_argument('--no-cpu-baseline', action='store_true')
    p.add_argument('--cpu-sample-z', type=int, default=1024)
    p.add_argument('--cold-child', default=None, help=argparse.SUPPRESS)   # internal: see cold_start()
    p.add_argument('--traffic-json', default=None,
                   help='tools/prof_summary.py output (rocprofv3 FETCH_SIZE / WRITE_SIZE passes) to fill '
                        'roofline.traffic; default profiles/traffic_<workload tag>.json when present')
    return p.parse_args(argv)


def launcher_cmd(gpus, argv, port, script=None):
    """The torch.distributed.run command that starts `gpus` ranks of this script with the same
    arguments (one process per GPU; rendezvous on 127.0.0.1)."""
    return [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', str(gpus),
            '--master-addr', '127.0.0.1', '--master-port', str(port),
            script or os.path.abspath(__file__)] + list(argv)


def needs_launch(gpus, env=None):
    """True when `--gpus N > 1` was asked for outside torch.distributed.run."""
    env = os.environ if env is None else env
    return gpus > 1 and 'WORLD_SIZE' not in env


def self_launch(gpus, argv):
    """Start the N ranks as a CHILD process (torch.distributed.run) and wait for it.  Runs before
    anything in this process touches torch or the GPU; the ranks inherit stdout, so rank 0's JSON
    line reaches the caller unchanged.  Returns the child's exit code (non-zero if any rank failed)."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    env = dict(os.environ)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')      # dmabuf IPC only on these hosts (RCCL)
    r = subprocess.run(launcher_cmd(gpus, argv, port), env=env)
    return r.returncode


def cpu_baseline(args, block_shape, shape_yx, nz):
    """Oracle C restatement of the reference target='local' path on host cores, on a bounded
    sample: the first `cpu_sample_z` planes of the same synthetic volume."""
    from oracle import oracle as O
    threads = int(os.environ.get('OMP_NUM_THREADS', '0')) or len(os.sched_getaffinity(0))
    threads = max(1, min(threads, 64))
    shape = (min(args.cpu_sample_z, nz),) + tuple(shape_yx)
    x = O.boundary_map(shape, n_threads=threads, dither=args.dither)
    t0 = time.perf_counter()
    r = O.label_volume(x, block_shape, args.threshold, args.mode, n_threads=threads, want_lut=False)
    dt = time.perf_counter() - t0
    nvox = x.size
    del x, r
    return {'value': round(nvox / dt / 1e9, 4), 'unit': 'Gvox/s', 'cores': threads, 'kind': 'port',
            'sample': 'oracle/cc_oracle.c (C restatement of the 5 reference stages, n_jobs=%d threads, '
                      'blocks strided as LocalTask) on shape %s block %s, %.2f s wall'
                      % (threads, list(shape), list(block_shape), dt)}


def cold_child(args):
    """Runs in a fresh process (cold_start): the input is read from a .npy file and uploaded,
    then the FIRST library call is timed -- context creation, code-object load on the first
    launch, workspace allocation, the kernels -- followed by warm calls.  Prints one JSON line."""
    import numpy as np
    import torch
    from cluster_tools_amd import _lib
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    x = torch.from_numpy(np.load(args.cold_child)).to(dev)
    out = torch.empty(x.shape, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    block_shape = tuple(int(v) for v in args.block_shape.split(','))
    t0 = time.perf_counter()
    ctx = _lib.Context(0)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    ctx.label_volume(x, block_shape, args.threshold, args.mode, out=out)
    torch.cuda.synchronize()
    cold = time.perf_counter() - t0
    host = {k: {'count': v['count'], 'ms': round(v['total_ms'], 3)} for k, v in ctx.profile().items()
            if k.startswith('host_')}
    warm = []
    for _ in range(5):
        t0 = time.perf_counter()
        ctx.label_volume(x, block_shape, args.threshold, args.mode, out=out)
        torch.cuda.synchronize()
        warm.append(time.perf_counter() - t0)
    ctx.close()
    print(json.dumps({'cold_ms': round(cold * 1e3, 3), 'warm_ms': round(min(warm) * 1e3, 3), 'first_call_host': host}),
          flush=True)


def cold_start(args, x, block_shape):
    """First-call cost of a one-shot job: `x` (the device input) goes to a .npy file, a child
    process (subprocess, not exec) runs cold_child on it."""
    import subprocess
    import tempfile
    import numpy as np
    with tempfile.TemporaryDirectory(prefix='cc_cold_') as d:
        path = os.path.join(d, 'x.npy')
        np.save(path, x.cpu().numpy())
        cmd = [sys.executable, os.path.abspath(__file__), '--cold-child', path, '--block-shape',
               ','.join(map(str, block_shape)), '--threshold', str(args.threshold), '--mode', args.mode]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        raise RuntimeError('cold-start child failed (%d): %s' % (r.returncode, r.stderr[-2000:]))
    if os.environ.get('CC_ALLOC_LOG'):
        sys.stderr.write(r.stderr)
    res = json.loads(r.stdout.strip().splitlines()[-1])
    res['how'] = ('fresh process: torch up and the input in HBM, then timed: cc_create + the first '
                  'cc_label_volume (code-object load, workspace allocation, kernels) to completion; '
                  'warm_ms = the best of the next 5 calls')
    return res


def load_traffic(path, kernel, lib_src):
    """Per-launch HBM bytes of `kernel` from a tools/prof_summary.py file (PMC passes, corrected as
    MI355X_MICROARCH.md §HBM says) -> (bytes or None, the file's lib_src).  The figure is used only
    when the file is stamped with the source hash of the library being benched: a stale figure
    never reaches the line."""
    if not os.path.exists(path):
        return None, None
    tdat = json.load(open(path))
    src = tdat.get('_meta', {}).get('lib_src')
    if src is None or src != lib_src:
        return None, src
    for k, v in tdat.items():
        if k.split('<')[0] == kernel and 'traffic' in v:
            return int(v['traffic']), src
    return None, src


def main():
    args = parse()
    if args.cold_child:
        return cold_child(args)
    if needs_launch(args.gpus):
        return self_launch(args.gpus, sys.argv[1:])
    import numpy as np
    import torch
    import torch.distributed as dist
    from cluster_tools_amd import _lib
    # the library must be built from this tree's sources (CC_LIB_PATH: another build for same-box
    # A/B timing, tools/ab_build.sh -- the line is then marked as such)
    lib_src = _lib.check_provenance() if not os.environ.get('CC_LIB_PATH') else 'override:' + _lib.LIB_PATH

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    assert world == args.gpus, 'launch N > 1 with torch.distributed.run (WORLD_SIZE must equal --gpus)'
    # CC_DIST_BACKEND=gloo: rehearsal of the N > 1 schedule with several ranks on one GPU (RCCL
    # refuses two ranks on one device); collectives staged through host memory
    backend = os.environ.get('CC_DIST_BACKEND', 'nccl')
    if world > 1:
        from cluster_tools_amd.distributed import check_rccl_ranks
        check_rccl_ranks(backend, local_rank, int(os.environ.get('LOCAL_WORLD_SIZE', world)))
    gpu = local_rank if backend == 'nccl' else local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(gpu)
    dev = torch.device('cuda', gpu)
    if world > 1:
        os.environ.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=dev)
        else:
            dist.init_process_group(backend)

    # workloads: strong = the volume is fixed and split into z-slabs over the N
    # ranks; weak = every rank owns a slab of the same size
    wl = args.workload
    spec = dict(WORKLOADS[wl])
    if args.mask:
        spec['mask'] = True
    block_shape = tuple(int(v) for v in (args.block_shape or ','.join(map(str, spec['block']))).split(','))
    from cluster_tools_amd.distributed import slab_bounds
    if args.shape:
        slab = tuple(int(v) for v in args.shape.split(','))
        gshape, z0, scaling = (slab[0] * world,) + slab[1:], slab[0] * rank, 'weak'
    elif spec['scaling'] == 'weak':
        slab = spec['per_rank']
        gshape, z0, scaling = (slab[0] * world,) + slab[1:], slab[0] * rank, 'weak'
    else:
        gshape = spec['shape']
        z0, zs = slab_bounds(gshape[0], block_shape[0], world)[rank]
        slab, scaling = (zs,) + tuple(gshape[1:]), 'strong'
    masked = bool(spec.get('mask'))
    tag = (wl if not args.shape else 'custom') + ('_mask' if masked and wl != 'c4' else '') + \
        ('_cont' if args.dither else '') + ('' if args.mode == 'greater' else '_' + args.mode) + \
        ('' if world == 1 else '_n%d' % world)
    workload = '%s%s%s %s f32, block %s, %s over %d GPU%s' % (
        wl.upper() if not args.shape else 'custom', ' + uint8 ellipsoid mask' if masked else '',
        ' continuous (dithered)' if args.dither else '', tuple(gshape), tuple(block_shape),
        '%s-scaled z-slabs' % scaling if world > 1 else 'one volume', world, 's' if world > 1 else '')

    ctx = _lib.Context(gpu)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    x = ctx.generate_boundary_map(slab, origin=(z0, 0, 0), device=dev, dither=args.dither)
    mask = None
    if masked:
        from cluster_tools_amd.synthetic import ellipsoid_mask_device
        mask = ellipsoid_mask_device(gshape, z0, slab[0], dev)
    out = torch.empty(slab, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()

    if world == 1:
        def step():
            return ctx.label_volume(x, block_shape, args.threshold, args.mode, mask=mask, out=out)[1]
    else:
        from cluster_tools_amd.distributed import ShardedLabeler, StagedComm
        comm = StagedComm(device=dev) if backend != 'nccl' else None
        lab = ShardedLabeler(ctx, gshape, block_shape, z0, slab[0], dev, comm=comm)

        def step():
            return lab.label(x, args.threshold, args.mode, mask=mask, out=out)

    for _ in range(args.warmup):
        res = step()
    # timed region: HIP events only around the volume-sized kernels (k_spec, k_pass2), so the
    # roofline kernel is timed live without an event pair around every small launch
    ctx.set_profiling(args.timed_prof)
    ctx.reset_profile()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    prof = ctx.profile()
    # per-kernel breakdown: the same steps again (untimed), an event pair around every launch
    ctx.set_profiling(1)
    ctx.reset_profile()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    breakdown = ctx.profile()
    ctx.set_profiling(False)
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev if backend == 'nccl' else 'cpu')
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    nvox_rank = int(np.prod(slab))
    nvox_all = int(np.prod(gshape))
    ms_per_step = dt / args.steps * 1e3
    value = nvox_all * args.steps / dt / 1e9
    b_alg = B_ALG + (1.0 if masked else 0.0)
    if masked:
        # input bytes only for the blocks holding a mask voxel (see live_voxels)
        lv = torch.tensor([float(live_voxels(mask, block_shape))], dtype=torch.float64,
                          device=dev if world > 1 and backend == 'nccl' else 'cpu')
        if world > 1:
            dist.all_reduce(lv)
        b_alg = round(8.0 + 1.0 + 4.0 * float(lv.item()) / nvox_all, 4)
    # dominant kernel of this rank, timed by HIP events on the stream it runs on
    # host_* entries are the library's host-side accounting (allocations, stream synchronisations)
    host = {k: v for k, v in breakdown.items() if k.startswith('host_')}
    prof = {k: v for k, v in prof.items() if not k.startswith('host_')}
    breakdown = {k: v for k, v in breakdown.items() if not k.startswith('host_')}
    kern = {k: v for k, v in prof.items() if v['count']}
    dom = max(kern, key=lambda k: kern[k]['total_ms'])
    avg_ms = kern[dom]['total_ms'] / kern[dom]['count']
    step_ms = kern[dom]['total_ms'] / args.steps      # == avg_ms for a kernel launched once per step
    kb = KERNEL_BYTES.get(dom)
    if dom == 'k_spec' and masked:
        kb += 1.0
    tj = args.traffic_json or os.path.join(ROOT, 'profiles', 'traffic_%s.json' % tag)
    traffic, traffic_src = load_traffic(tj, dom, lib_src)
    roofline = None
    if kb is not None:
        achieved = kb * nvox_rank / (step_ms * 1e-3) / 1e9
        roofline = {'bound': 'hbm', 'kernel': dom, 'achieved': round(achieved, 1), 'peak': HBM_PEAK_GBS,
                    'unit': 'GB/s', 'frac': round(achieved / HBM_PEAK_GBS, 4), 'traffic': traffic,
                    'traffic_file': {'path': os.path.relpath(tj, ROOT), 'lib_src': traffic_src,
                                     'used': traffic is not None} if os.path.exists(tj) else None,
                    'alg_bytes_per_voxel': kb, 'avg_launch_ms': round(avg_ms, 4),
                    'launches_per_step': kern[dom]['count'] / args.steps}
    e2e_gbs = b_alg * nvox_all * args.steps / dt / 1e9 / world

    line = {
        'metric': METRIC, 'value': round(value, 3), 'unit': 'Gvox/s', 'n_gpus': world,
        'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(ms_per_step, 3),
        'higher_is_better': True, 'scaling': scaling, 'vs_baseline': None, 'dtype': 'f32',
        'data': 'synthetic (integer-only jittered-Voronoi boundary map, SURVEY.md §8d, seed 0x5EED%s)'
                % (', + sub-2^-8 dither: continuous float32' if args.dither else ''),
        'config': {'workload': workload, 'workload_id': wl, 'shape': list(gshape), 'slab': list(slab),
                   'block_shape': list(block_shape), 'threshold': args.threshold,
                   'threshold_mode': args.mode, 'mask': masked, 'continuous': bool(args.dither),
                   'parallelism': 'z-slab x%d' % world if world > 1 else 'single GPU'},
        'roofline': roofline,
        'e2e_roofline': {'alg_bytes_per_voxel': b_alg, 'achieved_gbs_per_gpu': round(e2e_gbs, 1),
                         'frac': round(e2e_gbs / HBM_PEAK_GBS, 4)},
        'kernels_ms_per_step': {k: round(v['total_ms'] / args.steps, 4) for k, v in
                                sorted(breakdown.items(), key=lambda kv: -kv[1]['total_ms']) if v['count']},
        'host_per_step': {k: {'count': v['count'] / args.steps, 'ms': round(v['total_ms'] / args.steps, 4)}
                          for k, v in host.items()},
        'result': res,
        'lib': {'version': _lib.version(), 'src': lib_src},
    }
    if wl == 'c1' and world == 1:
        line['cold_start'] = cold_start(args, x, block_shape)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        del x, out
        torch.cuda.empty_cache()
        line['cpu_baseline'] = cpu_baseline(args, block_shape, slab[1:], slab[0])
    elif rank == 0:
        line['cpu_baseline'] = None
    if rank == 0:
        print(json.dumps(line), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    sys.exit(main() or 0)
