#!/opt/conda/bin/python3.9
"""Golden vectors for multi-channel input (`channel` parameter), from the REFERENCE's own jobs.

Run only in the build container (needs /root/reference and the conda python):

    /opt/conda/bin/python3.9 tests/golden/make_golden_channel.py

What runs: the five reference stages exactly as in make_golden.py, with `channel` in the
block_components job config (block_components.py:150-159: the selected channels of a 4-D
(C, Z, Y, X) dataset are copied into an array of the dataset's dtype and averaged with
np.mean(axis=0) before vu.normalize), and the reference `threshold` job with `channel`
(threshold.py:131-171, same averaging).  Inputs: float32 with channel magnitudes far apart (the
float32 summation order shows in the result), uint8 / uint16 / float64 (np.mean accumulates in
float64 for them), an int channel, repeated and reordered channel lists, a mask.

Output: tests/golden/channel_<case>.npz (input, channel list, the reference artefacts as in
make_golden.py, and `thr_expected` = the reference threshold job's uint8 output) and
tests/golden/index_channel.json.
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
from make_golden import canon, run_reference  # noqa: E402
import h5py  # noqa: E402
from cluster_tools.thresholded_components import threshold as ref_th  # noqa: E402
from oracle.synth import boundary_q, ellipsoid_mask  # noqa: E402


def run_reference_threshold(inp, block_shape, threshold, mode, channel, n_jobs=2, extra=None):
    tmp = tempfile.mkdtemp(prefix='golden_chthr_')
    try:
        in_path, out_path = os.path.join(tmp, 'in.h5'), os.path.join(tmp, 'out.h5')
        with h5py.File(in_path, 'w') as f:
            f.create_dataset('raw', data=inp)
        shape = inp.shape[1:] if channel is not None else inp.shape
        with h5py.File(out_path, 'w') as f:
            f.create_dataset('thr', shape=shape, dtype='uint8')
        nb = make_golden.n_blocks_of(shape, block_shape)
        for j in range(min(nb, n_jobs)):
            p = os.path.join(tmp, 'threshold_job_%i.config' % j)
            with open(p, 'w') as fh:
                json.dump({'input_path': in_path, 'input_key': 'raw', 'output_path': out_path,
                           'output_key': 'thr', 'block_list': list(range(nb))[j::n_jobs],
                           'block_shape': list(block_shape), 'threshold': float(threshold),
                           'threshold_mode': mode, 'channel': channel, **(extra or {})}, fh)
            ref_th.threshold(j, p)
        with h5py.File(out_path, 'r') as f:
            return f['thr'][:]
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def make_cases():
    rng = np.random.default_rng(20261016)
    cases = []

    def add(name, inp, channel, block_shape, threshold, mode, mask=None):
        cases.append(dict(name=name, inp=inp, channel=channel, block_shape=block_shape,
                          threshold=threshold, mode=mode, mask=mask))

    # float32, channel magnitudes far apart: (c_a + c_b) + c_c rounds differently by order
    f = rng.random((3, 12, 18, 24), dtype=np.float32)
    f[1] = f[1] * np.float32(1000.0) + np.float32(3.0)
    f[2] = f[2] * np.float32(1e-3) - np.float32(0.5)
    add('f32_int', f, 1, (4, 6, 8), 0.5, 'greater')
    add('f32_pair', f, [0, 2], (4, 6, 8), 0.45, 'less')
    add('f32_rep', f, [2, 1, 0, 1], (6, 9, 12), 0.5, 'greater')
    add('f32_rev', f, [1, 0, 2], (6, 9, 12), 0.5, 'greater')
    add('f32_mask', f, [0, 1], (4, 6, 8), 0.3, 'greater',
        mask=rng.choice(np.array([0, 1, 9], dtype=np.uint8), size=(12, 18, 24), p=[0.3, 0.4, 0.3]))
    # boundary-map-like channels: tile seams and block faces at the usual scale
    q = boundary_q((40, 72, 88))
    q2 = boundary_q((40, 72, 88), origin=(11, 3, 70))
    bm = np.stack([q.astype(np.float32) / np.float32(256), q2.astype(np.float32) / np.float32(256),
                   rng.random((40, 72, 88), dtype=np.float32) * np.float32(0.05)])
    add('bmap3', bm, [0, 1, 2], (16, 32, 32), 0.5, 'greater')
    add('bmap3_less_mask', bm, [0, 1], (16, 32, 32), 0.5, 'less', mask=ellipsoid_mask((40, 72, 88)))
    # integer and float64 inputs: np.mean accumulates in float64, normalize casts to float32
    u8 = rng.integers(0, 256, size=(2, 16, 24, 32)).astype(np.uint8)
    add('u8_pair', u8, [0, 1], (8, 12, 16), 0.5, 'greater')
    add('u8_equal', u8, [1, 0], (8, 12, 16), 0.5, 'equal')
    u16 = rng.integers(0, 65536, size=(5, 10, 14, 18)).astype(np.uint16)
    add('u16_five', u16, [4, 3, 2, 1, 0], (5, 7, 9), 0.6, 'less')
    f64 = rng.standard_normal((3, 10, 14, 18))
    f64[1] *= 1e6
    add('f64_pair', f64, [1, 2], (5, 7, 9), 0.5, 'greater')
    return cases


def main():
    index = {}
    for c in make_cases():
        res = run_reference(c['inp'], c['block_shape'], c['threshold'], c['mode'], mask=c['mask'],
                            channel=c['channel'])
        thr = run_reference_threshold(c['inp'], c['block_shape'], c['threshold'], c['mode'], c['channel'])
        chans = [c['channel']] if isinstance(c['channel'], int) else list(c['channel'])
        arrays = dict(
            input=c['inp'], channel=np.array(chans, dtype=np.int64),
            block_shape=np.array(c['block_shape'], dtype=np.int64),
            threshold=np.array(c['threshold'], dtype=np.float64),
            block_values=res['block_values'], offsets=res['offsets'],
            empty_blocks=res['empty_blocks'], n_labels=np.array(res['n_labels'], dtype=np.uint64),
            local_labels=res['local_labels'].astype(np.uint32), pairs=res['pairs'],
            lut_canon=canon(res['lut']), labels_canon=canon(res['labels']),
            max_id=np.array(res['max_id'], dtype=np.uint64), thr_expected=thr.astype(np.uint8))
        if c['mask'] is not None:
            arrays['mask'] = c['mask']
        np.savez_compressed(os.path.join(HERE, 'channel_%s.npz' % c['name']), **arrays)
        index[c['name']] = dict(shape=list(c['inp'].shape), dtype=str(c['inp'].dtype),
                                channel=c['channel'], block_shape=list(c['block_shape']),
                                threshold=c['threshold'], mode=c['mode'], mask=c['mask'] is not None,
                                n_components=int(arrays['labels_canon'].max()),
                                n_labels=int(res['n_labels']))
        print(c['name'], index[c['name']])
    with open(os.path.join(HERE, 'index_channel.json'), 'w') as fh:
        json.dump(index, fh, indent=1, sort_keys=True)


if __name__ == '__main__':
    main()
