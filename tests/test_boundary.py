"""The C-ABI boundary: the shared library loads without a GPU, exports every symbol the
header declares, and host-only entry points work.  CPU only."""
import os
import re

import numpy as np
import pytest

from conftest import ROOT


def header_functions(name='cc_mi355x.h'):
    src = open(os.path.join(ROOT, 'include', name)).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(cc_[a-z0-9_]+)\s*\(', src)))


def test_library_exports_every_declared_symbol():
    from cluster_tools_amd import _lib
    L = _lib.load()
    declared = header_functions()
    assert len(declared) >= 19
    for name in declared:
        assert hasattr(L, name), name
    assert set(declared) == set(_lib.EXPORTS)


def test_n5_library_exports_every_declared_symbol():
    from cluster_tools_amd import _lib
    L = _lib.load_n5()
    declared = header_functions('cc_n5.h')
    for name in declared:
        assert hasattr(L, name), name
    assert set(declared) == set(_lib.N5_EXPORTS)


def test_version_and_error_channel():
    from cluster_tools_amd import _lib
    L = _lib.load()
    assert b'gfx950' in L.cc_version()
    assert isinstance(L.cc_last_error(), bytes)


def test_merge_offsets_host_entry_matches_reference_rule():
    # merge_offsets.py:109-120 on a hand example: values n_i + 1 or 0
    from cluster_tools_amd import _lib
    values = np.array([3, 0, 5, 1, 0], dtype=np.uint64)
    offsets, empty, n_labels = _lib.merge_offsets(values)
    np.testing.assert_array_equal(offsets, [0, 3, 3, 8, 9])
    np.testing.assert_array_equal(empty, [1, 4])
    assert n_labels == 0 + 9 + 0 + 1  # offsets[-1] + values[-1] + 1 = 9 + 0 + 1


def test_no_silent_cpu_fallback_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip('GPU present')
    from cluster_tools_amd import _lib
    with pytest.raises(RuntimeError):
        _lib.Context(0)


def test_product_never_imports_oracle():
    pkg = os.path.join(ROOT, 'cluster_tools_amd')
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith('.py'):
                txt = open(os.path.join(dirpath, f)).read()
                for line in txt.splitlines():
                    s = line.strip()
                    if s.startswith('import') or s.startswith('from'):
                        assert 'oracle' not in s, (f, s)


@pytest.mark.parametrize('gshape,z0,nz', [((37, 20, 23), 0, 37), ((40, 16, 18), 10, 20)])
def test_device_mask_generator_matches_oracle(gshape, z0, nz):
    import torch
    from cluster_tools_amd.synthetic import ellipsoid_mask_device
    from oracle.synth import ellipsoid_mask
    got = ellipsoid_mask_device(gshape, z0, nz, torch.device('cpu'), chunk=7).numpy()
    ref = ellipsoid_mask(gshape)[z0:z0 + nz]
    assert np.array_equal(got, ref)


def test_binary_provenance():
    """The library in the tree was built from the tree's sources (cc_version's src= hash)."""
    from cluster_tools_amd import _lib, build
    assert _lib.check_provenance() == build.source_hash()


def test_integration_binding_struct_matches_library():
    """INTEGRATION.md's reference-side binding (run as written) declares struct cc_result with
    the library's size and field order (the documented _Res had 6 of 7 fields)."""
    import ctypes
    from conftest import exec_integration_binding
    from cluster_tools_amd import _lib
    ns = exec_integration_binding()           # its own assert compares with cc_result_size()
    L = _lib.load()
    assert ctypes.sizeof(ns['_Res']) == L.cc_result_size() == ctypes.sizeof(_lib.CCResult)
    assert [f for f, _ in ns['_Res']._fields_] == [f for f, _ in _lib.CCResult._fields_]
    hdr = open(os.path.join(ROOT, 'include', 'cc_mi355x.h')).read()
    body = hdr[hdr.index('typedef struct {'):hdr.index('} cc_result;')]
    fields = re.findall(r'(?:u?int64_t)\s+(\w+);', re.sub(r'/\*.*?\*/', '', body, flags=re.S))
    assert fields == [f for f, _ in _lib.CCResult._fields_]


def test_integration_blocks_compile():
    """Every python block of INTEGRATION.md is valid python."""
    from conftest import integration_blocks
    blocks = integration_blocks()
    assert len(blocks) >= 4
    for i, b in enumerate(blocks):
        compile(b, 'INTEGRATION.md#%d' % i, 'exec')


def test_resized_mask_rule_and_loader(tmp_path):
    """Masks of another shape (volume_utils.py:174-184): load_mask returns a ResizedMask instead of
    raising, and the oracle's nearest-neighbour rule on a hand example (2x upsampling repeats,
    2x downsampling takes the odd centres)."""
    from cluster_tools_amd import n5
    from cluster_tools_amd.utils import volume_utils as vu
    from oracle import oracle as O
    m = np.arange(8, dtype=np.uint8).reshape(2, 2, 2) % 3
    up = O.resize_mask_nearest(m, (4, 4, 4))
    np.testing.assert_array_equal(up, (m.repeat(2, 0).repeat(2, 1).repeat(2, 2) != 0).astype(np.uint8))
    big = np.random.default_rng(0).integers(0, 2, (6, 8, 10)).astype(np.uint8)
    np.testing.assert_array_equal(O.resize_mask_nearest(big, (3, 4, 5)), big[1::2, 1::2, 1::2])
    p = str(tmp_path / 'm.n5')
    with n5.open_file(p) as f:
        f.create_dataset('mask', data=big, chunks=(3, 4, 5), compression='gzip')
    r = vu.load_mask(p, 'mask', (12, 16, 20))
    assert isinstance(r, vu.ResizedMask) and r.mask_shape == (6, 8, 10) and r.shape == (12, 16, 20)
    assert not isinstance(vu.load_mask(p, 'mask', (6, 8, 10)), vu.ResizedMask)


def test_host_only_load_skips_torch_and_refuses_it_later():
    """_lib.load(host_only=True) (the drop-in's one-shot job processes: cc_merge_offsets,
    cc_label_volume_host) binds the library without importing torch; a torch import afterwards in
    that process is refused on the next load() instead of running two HIP runtimes side by side."""
    import subprocess
    import sys
    code = (
        "import sys\n"
        "from cluster_tools_amd import _lib\n"
        "import numpy as np\n"
        "_lib.load(host_only=True)\n"
        "offs, empty, n = _lib.merge_offsets(np.array([3, 0, 2], dtype=np.uint64))\n"
        "assert 'torch' not in sys.modules, 'host-only load imported torch'\n"
        "assert list(offs) == [0, 3, 3] and n == 6, (list(offs), n)\n"
        "import torch\n"
        "try:\n"
        "    _lib.load()\n"
        "except RuntimeError as e:\n"
        "    assert 'host-only' in str(e)\n"
        "else:\n"
        "    raise SystemExit('torch after a host-only load was not refused')\n"
        "print('ok')\n")
    r = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True, timeout=300,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0 and r.stdout.strip().endswith('ok'), r.stdout + r.stderr
