"""Build libcc_mi355x.so (hipcc, gfx950) and libcc_n5.so (host C++, zlib) in-tree.  Used by
__graft_entry__.build().

Binary provenance: the build embeds a SHA-256 of every source the libraries are built from
(csrc/*.hip, csrc/*.hpp, csrc/*.cpp, include/*.h) in cc_version() / cc_n5_version() ("... src=<hash>").
`source_hash()` recomputes it from the tree; `_lib.check_provenance()` compares the two, and
bench.py / the GPU tests refuse a library built from other sources than the tree's.
"""
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, 'csrc')
INCLUDE = os.path.join(os.path.dirname(HERE), 'include')
OUT = os.path.join(HERE, 'lib', 'libcc_mi355x.so')
OUT_N5 = os.path.join(HERE, 'lib', 'libcc_n5.so')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ARCH = os.environ.get('CC_OFFLOAD_ARCH', 'gfx950')
UNITS = ('cc_lib', 'cc_aux')      # translation units of libcc_mi355x.so


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(('.hip', '.hpp', '.cpp')))


def headers():
    return sorted(os.path.join(INCLUDE, f) for f in os.listdir(INCLUDE) if f.endswith('.h'))


def source_hash():
    """SHA-256 (first 16 hex digits) over the names and bytes of the libraries' sources."""
    h = hashlib.sha256()
    for p in sources() + headers():
        h.update(os.path.basename(p).encode() + b'\0')
        with open(p, 'rb') as f:
            h.update(f.read())
        h.update(b'\0')
    return h.hexdigest()[:16]


def needs_rebuild():
    if not os.path.exists(OUT) or not os.path.exists(OUT_N5):
        return True
    t = min(os.path.getmtime(OUT), os.path.getmtime(OUT_N5))
    return any(os.path.getmtime(s) > t for s in sources() + headers())


def build(force=False, verbose=True):
    if not force and not needs_rebuild():
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    h = '-DCC_SRC_HASH="%s"' % source_hash()
    cmd_n5 = [os.environ.get('CXX', 'g++'), '-O3', '-std=c++17', '-fPIC', '-shared', '-Wall', h,
              '-o', OUT_N5 + '.tmp', os.path.join(CSRC, 'cc_n5.cpp'), '-lz', '-pthread']
    # two translation units, two code objects (cc_aux.hip says why), compiled side by side
    flags = [HIPCC, '--offload-arch=%s' % ARCH, '-O3', '-std=c++17', '-fPIC', '-Wall', '-Wno-unused-function', h]
    objs = [OUT + '.%s.o' % u for u in UNITS]
    cmds = [flags + ['-c', os.path.join(CSRC, u + '.hip'), '-o', o] for u, o in zip(UNITS, objs)]
    if verbose:
        print(' '.join(cmd_n5), file=sys.stderr)
    subprocess.run(cmd_n5, check=True)
    os.replace(OUT_N5 + '.tmp', OUT_N5)
    procs = []
    for c in cmds:
        if verbose:
            print(' '.join(c), file=sys.stderr)
        procs.append(subprocess.Popen(c))
    rcs = [p.wait() for p in procs]
    if any(rcs):
        raise subprocess.CalledProcessError(max(rcs), cmds[rcs.index(max(rcs))])
    link = [HIPCC, '--offload-arch=%s' % ARCH, '-shared', '-o', OUT + '.tmp'] + objs
    if verbose:
        print(' '.join(link), file=sys.stderr)
    subprocess.run(link, check=True)
    for o in objs:
        os.remove(o)
    os.replace(OUT + '.tmp', OUT)
    return OUT


if __name__ == '__main__':
    build(force='--force' in sys.argv)
