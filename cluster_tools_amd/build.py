"""Build libcc_mi355x.so in-tree (hipcc, gfx950).  Used by __graft_entry__.build().

Binary provenance: the build embeds a SHA-256 of every source it is built from (csrc/*.hip,
csrc/*.hpp, csrc/*.cpp and include/cc_mi355x.h) in cc_version() ("... src=<hash>").
`source_hash()` recomputes it from the tree; `_lib.check_provenance()` compares the two, and
bench.py / the GPU tests refuse a library built from other sources than the tree's.
"""
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, 'csrc')
HEADER = os.path.join(os.path.dirname(HERE), 'include', 'cc_mi355x.h')
OUT = os.path.join(HERE, 'lib', 'libcc_mi355x.so')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ARCH = os.environ.get('CC_OFFLOAD_ARCH', 'gfx950')


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(('.hip', '.hpp', '.cpp')))


def source_hash():
    """SHA-256 (first 16 hex digits) over the names and bytes of the library's sources."""
    h = hashlib.sha256()
    for p in sources() + [HEADER]:
        h.update(os.path.basename(p).encode() + b'\0')
        with open(p, 'rb') as f:
            h.update(f.read())
        h.update(b'\0')
    return h.hexdigest()[:16]


def needs_rebuild():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(s) > t for s in sources() + [HEADER])


def build(force=False, verbose=True):
    if not force and not needs_rebuild():
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    cmd = [HIPCC, '--offload-arch=%s' % ARCH, '-O3', '-std=c++17', '-fPIC', '-shared',
           '-Wall', '-Wno-unused-function', '-DCC_SRC_HASH="%s"' % source_hash(),
           '-o', OUT + '.tmp', os.path.join(CSRC, 'cc_lib.hip'), '-lz']
    if verbose:
        print(' '.join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(OUT + '.tmp', OUT)
    return OUT


if __name__ == '__main__':
    build(force='--force' in sys.argv)
