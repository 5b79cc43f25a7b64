#!/opt/conda/bin/python3.9
"""Golden vectors for the Threshold task, from the REFERENCE's own job function.

Run only in the build container (needs /root/reference and the conda python):

    /opt/conda/bin/python3.9 tests/golden/make_golden_threshold.py

What runs: `threshold` (cluster_tools/thresholded_components/threshold.py:174-213, which calls
_threshold_block :131-171 -> vu.normalize volume_utils.py:98-105 and the float32 compare),
unmodified, with the same local stand-ins as make_golden.py (luigi, nifty blocking; storage
h5py instead of z5py), driven with a hand-written job config the way LocalTask writes it
(block_list[j::n_jobs], cluster_tasks.py:301-335).  Inputs are those of the labelling golden
cases (tests/golden/<case>.npz, no mask: the Threshold task has none).

Output: tests/golden/threshold_<case>.npz with `expected` (uint8, the reference output) and
the parameters; the input stays in <case>.npz.
"""
import json
import os
import shutil
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden  # noqa: E402  (registers the bare reference packages and the stubs)
import h5py  # noqa: E402
from cluster_tools.thresholded_components import threshold as ref_th  # noqa: E402

CASES = [  # (labelling case providing the input, block_shape, threshold, mode)
    ('bmap_greater', (16, 32, 32), 0.5, 'greater'),
    ('bmap_less', (16, 32, 32), 0.5, 'less'),
    ('bmap_equal_half', (16, 32, 32), 0.5, 'equal'),
    ('bmap_odd_blocks', (5, 7, 9), 0.5, 'greater'),
    ('noise_tiny_blocks', (4, 6, 8), 0.7, 'greater'),
    ('norm_edge_greater', (8, 12, 16), 0.5, 'greater'),
    ('norm_edge_less', (8, 12, 16), 0.5, 'less'),
    ('norm_edge_equal0', (8, 12, 16), 0.0, 'equal'),
    ('inf_block', (4, 12, 16), 0.4, 'less'),
    ('denormal_range', (4, 6, 8), 0.5, 'greater'),
    ('levels_equal_half', (4, 6, 8), 0.5, 'equal'),
    ('all_fg_const', (4, 6, 8), 0.5, 'less'),
]


def case_input(name):
    z = np.load(os.path.join(HERE, name + '.npz'))
    if 'input_q' in z:
        return z['input_q'].astype(np.float32) / np.float32(256)
    return z['input']


def run_reference_threshold(inp, block_shape, threshold, mode, n_jobs=2):
    tmp = tempfile.mkdtemp(prefix='golden_thr_')
    try:
        in_path, out_path = os.path.join(tmp, 'in.h5'), os.path.join(tmp, 'out.h5')
        with h5py.File(in_path, 'w') as f:
            f.create_dataset('raw', data=inp)
        with h5py.File(out_path, 'w') as f:
            f.require_dataset('thr', shape=inp.shape, dtype='uint8', compression='gzip',
                              chunks=tuple(min(b, s) for b, s in zip(block_shape, inp.shape)))
        nb = make_golden.n_blocks_of(inp.shape, block_shape)
        for j in range(min(nb, n_jobs)):
            cfg = {'input_path': in_path, 'input_key': 'raw', 'output_path': out_path,
                   'output_key': 'thr', 'block_shape': list(block_shape),
                   'block_list': list(range(nb))[j::n_jobs], 'threshold': float(threshold),
                   'threshold_mode': mode, 'tmp_folder': tmp}
            p = os.path.join(tmp, 'threshold_job_%i.config' % j)
            with open(p, 'w') as fh:
                json.dump(cfg, fh)
            ref_th.threshold(j, p)
        with h5py.File(out_path, 'r') as f:
            return f['thr'][:]
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def main():
    for src, bs, t, mode in CASES:
        inp = case_input(src)
        exp = run_reference_threshold(inp, bs, t, mode)
        np.savez_compressed(os.path.join(HERE, 'threshold_%s.npz' % src), expected=exp,
                            block_shape=np.array(bs, dtype=np.int64),
                            threshold=np.array(t, dtype=np.float64), mode=np.array(mode))
        print(src, bs, t, mode, 'foreground', int(exp.sum()), 'of', exp.size)


if __name__ == '__main__':
    main()
