"""First-launch cost of a code object vs its kernel count and code size (tools only).

Generates libraries of N kernels (each with R unrolled rounds of integer work, to set the code
size), builds them here with hipcc (`build`), and on the GPU box times, in a fresh process per
library, dlopen + the first launch of kernel 0 + sync, then a second launch (`run`).
Prints one JSON line per library.

    python tools/cold_kernels.py build          # in the container
    python tools/cold_kernels.py run            # on the GPU box
"""
import ctypes
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, '_cold')
VARIANTS = [(1, 1), (16, 1), (64, 1), (160, 1), (16, 64), (160, 16), (24, 2048)]


def source(n, reps):
    k = []
    for i in range(n):
        body = '\n'.join('        x = x * %du + (x >> %d) + p[(x + %d) & 63];' % (2 * j + 3 + i, 1 + j % 7, j)
                         for j in range(reps))
        k.append('__global__ void k%d(unsigned* p) {\n    unsigned x = threadIdx.x;\n'
                 '    for (int i = 0; i < (int)p[1]; ++i) {\n%s\n    }\n    p[2 + (threadIdx.x & 7)] = x;\n}\n'
                 % (i, body))
    return ('#include <hip/hip_runtime.h>\n' + ''.join(k) +
            'extern "C" int probe_launch(void* s, unsigned* p) {\n'
            '    hipLaunchKernelGGL(k0, dim3(1), dim3(64), 0, (hipStream_t)s, p);\n'
            '    return (int)hipGetLastError();\n}\n')


def name(n, reps):
    return os.path.join(OUT, 'libcold_%d_%d.so' % (n, reps))


def build():
    os.makedirs(OUT, exist_ok=True)
    for n, reps in VARIANTS:
        src = os.path.join(OUT, 'cold_%d_%d.hip' % (n, reps))
        with open(src, 'w') as f:
            f.write(source(n, reps))
        subprocess.run(['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-O3', '-shared', '-fPIC',
                        '-o', name(n, reps), src], check=True)
        print(name(n, reps), os.path.getsize(name(n, reps)), file=sys.stderr)


def child(path):
    import torch
    dev = torch.device('cuda', 0)
    a = torch.zeros(64, dtype=torch.int32, device=dev)
    a.add_(1)
    torch.cuda.synchronize()
    st = torch.cuda.current_stream(dev).cuda_stream
    r = {'lib': os.path.basename(path), 'bytes': os.path.getsize(path)}
    t0 = time.perf_counter()
    L = ctypes.CDLL(path)
    L.probe_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    r['dlopen_ms'] = (time.perf_counter() - t0) * 1e3
    for k in ('first_ms', 'second_ms'):
        t0 = time.perf_counter()
        assert L.probe_launch(st, a.data_ptr()) == 0
        torch.cuda.synchronize()
        r[k] = (time.perf_counter() - t0) * 1e3
    print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)


def run():
    for n, reps in VARIANTS:
        for _ in range(2):
            subprocess.run([sys.executable, __file__, 'child', name(n, reps)], check=True, timeout=120)


if __name__ == '__main__':
    {'build': build, 'run': run, 'child': lambda: child(sys.argv[2])}[sys.argv[1]]()
