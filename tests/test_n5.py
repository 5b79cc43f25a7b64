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
