"""Cold-start probe: in a fresh process with torch's queue already warm,
time (1) the first launch from a one-kernel library (tools/cold_probe.hip -> tools/libcold_probe.so)
and (2) ctx creation + the first and second cc_label_volume on a small volume.  The difference
between the two first launches is the cost of loading libcc_mi355x.so's code object.
Prints one JSON line."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from cluster_tools_amd import _lib
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    a = torch.zeros(16, dtype=torch.int32, device=dev)
    a.add_(1)
    torch.cuda.synchronize()
    st = torch.cuda.current_stream(dev).cuda_stream
    r = {}
    t0 = time.perf_counter()
    P = ctypes.CDLL(os.path.join(ROOT, 'tools', 'libcold_probe.so'))
    P.probe_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    r['probe_dlopen_ms'] = (time.perf_counter() - t0) * 1e3
    for k in ('probe_first_ms', 'probe_second_ms'):
        t0 = time.perf_counter()
        assert P.probe_launch(st, a.data_ptr()) == 0
        torch.cuda.synchronize()
        r[k] = (time.perf_counter() - t0) * 1e3
    lib = sys.argv[sys.argv.index('--lib') + 1] if '--lib' in sys.argv else None
    t0 = time.perf_counter()
    if lib:     # another build of the library (experiments): the three entry points only
        L = ctypes.CDLL(lib)
        P = ctypes.c_void_p
        L.cc_create.argtypes = [ctypes.c_int, ctypes.POINTER(P)]
        L.cc_set_stream.argtypes = [P, P]
        L.cc_label_volume.argtypes = [P, P, P, P, P, ctypes.c_double, ctypes.c_int, P, P]
        L.cc_destroy.argtypes = [P]
        L.cc_destroy.restype = None
    else:
        _lib.load()
    r['lib_dlopen_ms'] = (time.perf_counter() - t0) * 1e3
    t0 = time.perf_counter()
    if lib:
        h = ctypes.c_void_p()
        assert L.cc_create(0, ctypes.byref(h)) == 0
        L.cc_set_stream(h, st)
    else:
        ctx = _lib.Context(0)
        ctx.set_stream(st)
    torch.cuda.synchronize()
    r['ctx_create_ms'] = (time.perf_counter() - t0) * 1e3
    # --c1: the C1 geometry (125, 1250, 1250) block (50, 512, 512); uniform random input
    shape, bs = ((125, 1250, 1250), (50, 512, 512)) if '--c1' in sys.argv else ((64, 128, 128), (32, 64, 64))
    if '--host-input' in sys.argv:     # as bench.py's cold child: the input uploaded from host memory
        import numpy as np
        x = torch.from_numpy(np.random.default_rng(0).random(shape, dtype=np.float32)).to(dev)
    else:
        x = torch.rand(shape, dtype=torch.float32, device=dev)
    out = torch.empty(shape, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    import numpy as np
    shp, bsh = np.array(shape, dtype=np.int64), np.array(bs, dtype=np.int64)
    res = (ctypes.c_char * 4096)()
    for k in ('label_first_ms', 'label_second_ms', 'label_third_ms'):
        t0 = time.perf_counter()
        if lib:
            assert L.cc_label_volume(h, x.data_ptr(), None, shp.ctypes.data, bsh.ctypes.data, 0.5, 0,
                                     out.data_ptr(), ctypes.addressof(res)) == 0
        else:
            ctx.label_volume(x, bs, 0.5, 'greater', out=out)
        torch.cuda.synchronize()
        r[k] = (time.perf_counter() - t0) * 1e3
    t0 = time.perf_counter()
    if lib:
        L.cc_destroy(h)
    else:
        ctx.close()
    r['destroy_ms'] = (time.perf_counter() - t0) * 1e3
    r['env'] = {k: os.environ[k] for k in os.environ if k.startswith(('HIP_', 'AMD_', 'CC_'))}
    print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()}))


if __name__ == '__main__':
    main()
