"""Build libcc_mi355x.so in-tree (hipcc, gfx950).  Used by __graft_entry__.build()."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, 'csrc')
OUT = os.path.join(HERE, 'lib', 'libcc_mi355x.so')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ARCH = os.environ.get('CC_OFFLOAD_ARCH', 'gfx950')


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(('.hip', '.hpp')))


def needs_rebuild():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    hdr = os.path.join(os.path.dirname(HERE), 'include', 'cc_mi355x.h')
    return any(os.path.getmtime(s) > t for s in sources() + [hdr])


def build(force=False, verbose=True):
    if not force and not needs_rebuild():
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    cmd = [HIPCC, '--offload-arch=%s' % ARCH, '-O3', '-std=c++17', '-fPIC', '-shared',
           '-Wall', '-Wno-unused-function', '-o', OUT + '.tmp', os.path.join(CSRC, 'cc_lib.hip')]
    if verbose:
        print(' '.join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(OUT + '.tmp', OUT)
    return OUT


if __name__ == '__main__':
    build(force='--force' in sys.argv)
