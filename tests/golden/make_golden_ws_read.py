#!/opt/conda/bin/python3.9
"""Golden vectors for the watershed's 4-D (channel) input, from the REFERENCE's own `_read_data`
(cluster_tools/watershed/watershed_from_seeds.py:127-139), numpy only.

Run only in the build container (needs /root/reference and the conda python):

    /opt/conda/bin/python3.9 tests/golden/make_golden_ws_read.py

What runs: the reference module is imported with the stand-ins of make_golden.py (luigi, nifty,
...); for every block of the blocking, `_read_data(ds_in, bb, config)` reads the block of an h5
dataset (C, Z, Y, X): channels channel_begin:channel_end, vu.normalize of the 4-D block, then
np.mean / max / min over the channels (agglomerate_channels).  The per-block outputs are assembled
into the (Z, Y, X) float32 volume the watershed grows over.  Cases: the three aggregations,
channel ranges (open end, a sub-range), float32 channels with magnitudes far apart (the float32
summation order shows), uint8 / uint16 input (cast to float32 by normalize), a NaN voxel in one
block, a constant block, an inf voxel, odd edge blocks.

Output: tests/golden/ws_read_<case>.npz (input, block_shape, channel_begin/end, agg, expected)
and tests/golden/index_ws_read.json.
"""
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden  # noqa: E402  (registers the bare reference packages and the stubs)
from make_golden import _bare_package, REF  # noqa: E402
import h5py  # noqa: E402

_bare_package('cluster_tools.watershed', os.path.join(REF, 'cluster_tools', 'watershed'))
from cluster_tools.watershed import watershed_from_seeds as ref_ws  # noqa: E402
from oracle.synth import boundary_q  # noqa: E402


def blocks(shape, block_shape):
    Z, Y, X = shape
    bz, by, bx = block_shape
    for z0 in range(0, Z, bz):
        for y0 in range(0, Y, by):
            for x0 in range(0, X, bx):
                yield np.s_[z0:min(z0 + bz, Z), y0:min(y0 + by, Y), x0:min(x0 + bx, X)]


def run(x4, block_shape, cb, ce, agg):
    config = {'channel_begin': cb, 'channel_end': ce, 'agglomerate_channels': agg}
    out = np.zeros(x4.shape[1:], dtype=np.float32)
    with tempfile.TemporaryDirectory(prefix='golden_wsread_') as d:
        p = os.path.join(d, 'in.h5')
        with h5py.File(p, 'w') as f:
            f.create_dataset('raw', data=x4)
        with h5py.File(p, 'r') as f:
            ds = f['raw']
            for bb in blocks(x4.shape[1:], block_shape):
                r = ref_ws._read_data(ds, bb, config)
                assert r.dtype == np.float32, r.dtype
                out[bb] = r
    return out


def main():
    rng = np.random.default_rng(20261017)
    shape, bs = (20, 36, 44), (8, 16, 20)
    base = [boundary_q(shape, origin=(0, 3 * c, 5 * c)).astype(np.float32) / 256 for c in range(4)]
    cases = {}
    x = np.stack(base)
    cases['mean_all'] = (x, bs, 0, None, 'mean')
    cases['max_all'] = (x, bs, 0, None, 'max')
    cases['min_all'] = (x, bs, 0, None, 'min')
    cases['mean_sub'] = (x, bs, 1, 3, 'mean')
    cases['max_open_end'] = (x, bs, 2, None, 'max')
    far = x.copy()
    far[0] *= np.float32(1e6)
    far[1] = far[1] * np.float32(3e-3) + np.float32(0.1)
    far[2] += rng.standard_normal(shape).astype(np.float32) * np.float32(1e-4)
    cases['mean_far'] = (far, bs, 0, None, 'mean')
    u8 = (x * 255).astype(np.uint8)
    cases['mean_u8'] = (u8, bs, 0, 3, 'mean')
    u16 = (x * 60000).astype(np.uint16)
    cases['min_u16'] = (u16, bs, 1, None, 'min')
    special = x.copy()
    special[1, 3, 5, 7] = np.nan                   # one NaN voxel: its whole 4-D block is NaN
    special[:, 8:16, 16:32, 0:20] = np.float32(0.25)   # a constant block (max == 0: no division)
    special[2, 17, 30, 41] = np.inf                # +inf in an edge block
    for agg in ('mean', 'max', 'min'):
        cases['special_' + agg] = (special, bs, 0, None, agg)
    index = {}
    for name, (x4, block_shape, cb, ce, agg) in cases.items():
        exp = run(x4, block_shape, cb, ce, agg)
        np.savez_compressed(os.path.join(HERE, 'ws_read_%s.npz' % name), input=x4, expected=exp)
        index[name] = {'block_shape': list(block_shape), 'channel_begin': cb, 'channel_end': ce, 'agg': agg,
                       'dtype': str(x4.dtype), 'shape': list(x4.shape)}
        print(name, x4.dtype, x4.shape, 'nan' if np.isnan(exp).any() else '')
    with open(os.path.join(HERE, 'index_ws_read.json'), 'w') as f:
        json.dump(index, f, indent=1, sort_keys=True)


if __name__ == '__main__':
    main()
