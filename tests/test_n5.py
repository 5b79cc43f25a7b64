"""N5 container I/O (cluster_tools_amd/n5.py).  Byte layout follows the N5 spec; no z5py file
is available to pin it ('parity unpinned')."""
import gzip
import json
import os
import struct

import numpy as np

from cluster_tools_amd import n5


def test_roundtrip_and_partial_writes(tmp_path):
    p = str(tmp_path / 'data.n5')
    a = (np.arange(13 * 17 * 19) % 251).reshape(13, 17, 19).astype('uint64') * 1234567
    with n5.open_file(p) as f:
        ds = f.create_dataset('g/seg', shape=a.shape, dtype='uint64', chunks=(4, 8, 5), compression='gzip')
        ds[:] = a
        ds[3:9, 2:11, 7:18] = a[3:9, 2:11, 7:18] + 1
        ds.attrs['maxId'] = 42
    with n5.open_file(p, 'r') as f:
        ds = f['g/seg']
        b = ds[:]
        assert ds.attrs['maxId'] == 42
        assert ds.chunks == (4, 8, 5) and ds.shape == a.shape
    ref = a.copy()
    ref[3:9, 2:11, 7:18] += 1
    np.testing.assert_array_equal(b, ref)


def test_spec_layout(tmp_path):
    """attributes are fastest-first; chunk path <x>/<y>/<z>; big-endian header and payload."""
    p = str(tmp_path / 'x.n5')
    a = np.arange(2 * 3 * 4, dtype='float32').reshape(2, 3, 4)
    with n5.open_file(p) as f:
        f.create_dataset('raw', data=a, chunks=(2, 2, 3), compression='gzip')
    meta = json.load(open(os.path.join(p, 'raw', 'attributes.json')))
    assert meta['dimensions'] == [4, 3, 2] and meta['blockSize'] == [3, 2, 2]
    assert meta['dataType'] == 'float32' and meta['compression']['type'] == 'gzip'
    assert json.load(open(os.path.join(p, 'attributes.json')))['n5']
    # chunk (z=0, y=1, x=1) = a[0:2, 2:3, 3:4] -> file raw/1/1/0, truncated edge chunk
    buf = open(os.path.join(p, 'raw', '1', '1', '0'), 'rb').read()
    mode, ndim = struct.unpack('>HH', buf[:4])
    dims = struct.unpack('>III', buf[4:16])
    assert (mode, ndim, dims) == (0, 3, (1, 1, 2))
    vals = np.frombuffer(gzip.decompress(buf[16:]), dtype='>f4')
    np.testing.assert_array_equal(vals, a[0:2, 2:3, 3:4].ravel())


def test_missing_chunks_read_as_zero(tmp_path):
    p = str(tmp_path / 'y.n5')
    with n5.open_file(p) as f:
        ds = f.require_dataset('seg', shape=(10, 10, 10), dtype='uint64', chunks=(5, 5, 5))
        ds[0:5, 0:5, 0:5] = 7
        assert ds[:].sum() == 7 * 125


def _write_chunk_py(path, data, mode=0, full_dims=None):
    """An N5 chunk written independently of the library (python gzip + struct, N5 spec)."""
    import gzip as gz
    os.makedirs(os.path.dirname(path), exist_ok=True)
    dims = full_dims or data.shape
    head = struct.pack('>HH', mode, data.ndim) + struct.pack('>' + 'I' * data.ndim, *dims[::-1])
    if mode == 1:
        head += struct.pack('>I', data.size)
    with open(path, 'wb') as f:
        f.write(head + gz.compress(np.ascontiguousarray(data, dtype=data.dtype.newbyteorder('>')).tobytes()))


def test_native_reads_independently_written_chunks(tmp_path):
    """Chunks written by python's gzip module (default mode, varlength mode, a full-size edge chunk)
    decode through the native codec."""
    p = str(tmp_path / 'z.n5')
    with n5.open_file(p) as f:
        ds = f.create_dataset('v', shape=(5, 6, 7), dtype='uint32', chunks=(4, 4, 4), compression='gzip')
    a = (np.arange(5 * 6 * 7, dtype='uint32') * 2654435761 % 1000003).reshape(5, 6, 7)
    root = os.path.join(p, 'v')
    _write_chunk_py(os.path.join(root, '0', '0', '0'), a[0:4, 0:4, 0:4])
    _write_chunk_py(os.path.join(root, '1', '0', '0'), a[0:4, 0:4, 4:7], mode=1)
    full = np.zeros((4, 4, 4), dtype='uint32')
    full[:1, :2, :3] = a[4:5, 4:6, 4:7]
    _write_chunk_py(os.path.join(root, '1', '1', '1'), full, full_dims=(4, 4, 4))
    got = ds[:]
    ref = np.zeros_like(a)
    ref[0:4, 0:4, 0:7] = a[0:4, 0:4, 0:7]
    ref[4:5, 4:6, 4:7] = a[4:5, 4:6, 4:7]
    np.testing.assert_array_equal(got, ref)


def test_one_and_four_dimensional_datasets(tmp_path):
    p = str(tmp_path / 'w.n5')
    lut = (np.arange(100003, dtype=np.uint64) * 7) ^ np.uint64(1 << 40)
    x4 = np.random.default_rng(1).random((3, 9, 10, 11)).astype(np.float32)
    with n5.open_file(p) as f:
        f.create_dataset('assignments', data=lut, chunks=(65334,), compression='gzip')
        f.create_dataset('raw4', data=x4, chunks=(1, 4, 5, 6), compression='raw')
    with n5.open_file(p, 'r') as f:
        np.testing.assert_array_equal(f['assignments'][:], lut)
        np.testing.assert_array_equal(f['assignments'][65000:70000], lut[65000:70000])
        np.testing.assert_array_equal(f['raw4'][1:3, 2:9, :, 5:11], x4[1:3, 2:9, :, 5:11])
    # raw chunk payload is big-endian float32 after a 4 + 4*4 byte header
    buf = open(os.path.join(p, 'raw4', '0', '0', '0', '0'), 'rb').read()
    np.testing.assert_array_equal(np.frombuffer(buf[20:], dtype='>f4').reshape(1, 4, 5, 6), x4[0:1, 0:4, 0:5, 0:6])


def test_skip_zero_chunks_and_overwrite(tmp_path):
    """All-zero chunks are not created (the reference never writes empty blocks), but an existing
    chunk that becomes zero is rewritten."""
    p = str(tmp_path / 's.n5')
    with n5.open_file(p) as f:
        ds = f.create_dataset('seg', shape=(8, 8, 8), dtype='uint64', chunks=(4, 4, 4), compression='gzip')
        a = np.zeros((8, 8, 8), dtype=np.uint64)
        a[0, 0, 0] = 5
        ds.write_region([(0, 8)] * 3, a, skip_zero_chunks=True)
        assert ds.chunk_exists((0, 0, 0)) and not ds.chunk_exists((1, 1, 1))
        ds.write_region([(0, 8)] * 3, np.zeros_like(a), skip_zero_chunks=True)
        assert ds.chunk_exists((0, 0, 0))
        assert ds[:].sum() == 0


def test_threads_give_identical_files(tmp_path):
    a = np.random.default_rng(2).integers(0, 50, (37, 41, 43)).astype(np.uint64)
    blobs = []
    for nt in (1, 7):
        p = str(tmp_path / ('t%d.n5' % nt))
        with n5.open_file(p) as f:
            ds = f.create_dataset('seg', shape=a.shape, dtype='uint64', chunks=(8, 16, 16), compression='gzip')
            ds.n_threads = nt
            ds[:] = a
            np.testing.assert_array_equal(ds[:], a)
        blobs.append(open(os.path.join(p, 'seg', '2', '1', '4'), 'rb').read())
    assert blobs[0] == blobs[1]


def test_corrupt_chunk_raises(tmp_path):
    import pytest
    p = str(tmp_path / 'c.n5')
    with n5.open_file(p) as f:
        ds = f.create_dataset('seg', shape=(4, 4, 4), dtype='uint64', chunks=(4, 4, 4), compression='gzip')
        ds[:] = 1
    path = os.path.join(p, 'seg', '0', '0', '0')
    buf = open(path, 'rb').read()
    open(path, 'wb').write(buf[:-9])
    with pytest.raises(RuntimeError):
        n5.open_file(p, 'r')['seg'][:]


def _raw_chunk(path, mode, dims_fastest_first, payload, count=None):
    """A chunk file with an arbitrary (possibly lying) header, raw payload."""
    os.makedirs(os.path.dirname(path), exist_ok=True)
    head = struct.pack('>HH', mode, len(dims_fastest_first)) + struct.pack('>' + 'I' * len(dims_fastest_first),
                                                                          *dims_fastest_first)
    if mode == 1:
        head += struct.pack('>I', count)
    with open(path, 'wb') as f:
        f.write(head + payload)


def test_malformed_chunk_headers_raise(tmp_path):
    """Chunk headers are untrusted input: unknown modes, dims beyond the dataset's
    chunk size, a varlength count that differs from the dims, and a chunk smaller than its box
    must raise -- never index past the decoded array -- for reads and for the read-merge-rewrite
    of a partial write."""
    import pytest
    p = str(tmp_path / 'm.n5')
    with n5.open_file(p) as f:
        ds = f.create_dataset('v', shape=(8, 8, 8), dtype='uint32', chunks=(4, 4, 4), compression='raw')
    chunk = os.path.join(p, 'v', '0', '0', '0')
    full = np.arange(64, dtype='>u4').tobytes()
    cases = [
        (2, (4, 4, 4), full, None),                    # object mode: not a numeric chunk
        (0, (4, 4, 0x10000), full, None),              # dims beyond the chunk size
        (0, (0xFFFFFFFF, 0xFFFFFFFF, 4), full, None),  # product would overflow
        (1, (4, 4, 4), full[:16], 4),                  # varlength count != prod(dims)
        (0, (4, 2, 4), full[:128], None),              # smaller than its (4, 4, 4) box
    ]
    for mode, dims, payload, count in cases:
        _raw_chunk(chunk, mode, dims, payload, count)
        with pytest.raises(RuntimeError):
            ds[0:4, 0:4, 0:4]
        with pytest.raises(RuntimeError):             # partial write: read-merge-rewrite
            ds[1:3, 1:3, 1:3] = np.ones((2, 2, 2), dtype='uint32')
    # a well-formed varlength chunk still reads
    _raw_chunk(chunk, 1, (4, 4, 4), full, 64)
    np.testing.assert_array_equal(ds[0:4, 0:4, 0:4].ravel(), np.arange(64, dtype='uint32'))


def test_temp_names_differ_across_processes(tmp_path):
    """Two processes writing the same chunk use distinct temp files (pid in the name)."""
    import subprocess
    import sys
    p = str(tmp_path / 'r.n5')
    with n5.open_file(p) as f:
        f.create_dataset('seg', shape=(64, 64, 64), dtype='uint64', chunks=(64, 64, 64), compression='gzip')
    code = ('import sys, numpy as np; sys.path.insert(0, %r); from cluster_tools_amd import n5\n'
            'ds = n5.open_file(%r)["seg"]\n'
            'for i in range(20): ds[:] = np.full((64, 64, 64), int(sys.argv[1]), dtype=np.uint64)\n'
            % (os.path.dirname(os.path.dirname(os.path.abspath(__file__))), p))
    procs = [subprocess.Popen([sys.executable, '-c', code, str(k)]) for k in (3, 5)]
    assert all(q.wait(timeout=120) == 0 for q in procs)
    v = n5.open_file(p, 'r')['seg'][:]
    assert len(np.unique(v)) == 1 and int(v[0, 0, 0]) in (3, 5)
