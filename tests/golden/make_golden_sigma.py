#!/opt/conda/bin/python3.9
"""Golden vectors for sigma_prefilter > 0, from the REFERENCE's own jobs -- with the filter itself
restated.

Run only in the build container (needs /root/reference and the conda python):

    /opt/conda/bin/python3.9 tests/golden/make_golden_sigma.py

What runs: the five reference stages as in make_golden.py and the reference `threshold` job, with
`sigma_prefilter` in the job configs (block_components.py:160-163, threshold.py:150-153: per block
vu.normalize -> vu.apply_filter(., 'gaussianSmoothing', sigma) -> vu.normalize, then threshold,
mask, label).  The filter library is absent here (fastfilters, vigra): vu.apply_filter falls back to
the stand-in module vigra.filters (tests/golden/stubs), whose gaussianSmoothing is set to
oracle.gaussian_smooth -- the restatement of vigra's algorithm.  So these vectors pin everything
around the filter (the per-block composition, both normalizations with NaN / inf / constant
blocks, the float32 compare, the mask order, the labelling and merging) to the reference's own
code; the filter arithmetic itself stays unpinned against vigra.

Output: tests/golden/sigma_<case>.npz and tests/golden/index_sigma.json.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden  # noqa: E402  (registers the bare reference packages and the stubs)
from make_golden import canon, run_reference  # noqa: E402
from make_golden_channel import run_reference_threshold  # noqa: E402
import vigra.filters  # noqa: E402  (the stand-in module)
from oracle import oracle as O  # noqa: E402
from oracle.synth import boundary_q, ellipsoid_mask  # noqa: E402

vigra.filters.gaussianSmoothing = O.gaussian_smooth


def make_cases():
    rng = np.random.default_rng(20261017)
    cases = []

    def add(name, inp, block_shape, threshold, mode, sigma, mask=None, channel=None):
        cases.append(dict(name=name, inp=inp, block_shape=block_shape, threshold=threshold, mode=mode,
                          sigma=sigma, mask=mask, channel=channel))

    bm = boundary_q((40, 72, 88)).astype(np.float32) / np.float32(256)
    add('bmap_s1', bm, (16, 32, 32), 0.5, 'greater', 1.0)
    add('bmap_s2_less', bm, (16, 32, 32), 0.45, 'less', 2.0)
    add('bmap_s07_mask', bm, (16, 32, 32), 0.5, 'greater', 0.7, mask=ellipsoid_mask((40, 72, 88)))
    wn = rng.random((12, 18, 24), dtype=np.float32)
    add('noise_s05', wn, (6, 9, 12), 0.5, 'greater', 0.5)
    add('noise_s1_less', wn, (6, 9, 12), 0.5, 'less', 1.0)
    # normalisation edge cases around the filter: affine-rescaled, constant, NaN, +-inf blocks
    sm = rng.random((16, 24, 32), dtype=np.float32)
    sm[:8, :12, :16] = sm[:8, :12, :16] * np.float32(1000.0) + np.float32(5.0)
    sm[:8, 12:, :16] = np.float32(0.3)
    sm[8:, :12, 16:] = np.float32(np.nan)
    sm[9, 3, 5] = np.float32(np.nan)
    sm[2, 20, 20] = np.float32(np.inf)
    sm[12, 20, 4] = np.float32(-np.inf)
    add('norm_edge_s1', sm, (8, 12, 16), 0.5, 'greater', 1.0)
    add('norm_edge_s1_equal0', sm, (8, 12, 16), 0.0, 'equal', 1.0)
    # with channels (mean first, then the filter)
    f = rng.random((2, 12, 18, 24), dtype=np.float32)
    add('chan_s1', f, (6, 9, 12), 0.5, 'greater', 1.0, channel=[1, 0])
    return cases


def main():
    index = {}
    for c in make_cases():
        res = run_reference(c['inp'], c['block_shape'], c['threshold'], c['mode'], mask=c['mask'],
                            channel=c['channel'], extra={'sigma_prefilter': c['sigma']})
        thr = run_reference_threshold(c['inp'], c['block_shape'], c['threshold'], c['mode'], c['channel'],
                                      extra={'sigma_prefilter': c['sigma']})
        arrays = dict(
            input=c['inp'], sigma=np.array(c['sigma'], dtype=np.float64),
            block_shape=np.array(c['block_shape'], dtype=np.int64),
            threshold=np.array(c['threshold'], dtype=np.float64),
            block_values=res['block_values'], offsets=res['offsets'],
            empty_blocks=res['empty_blocks'], n_labels=np.array(res['n_labels'], dtype=np.uint64),
            local_labels=res['local_labels'].astype(np.uint32), pairs=res['pairs'],
            lut_canon=canon(res['lut']), labels_canon=canon(res['labels']),
            max_id=np.array(res['max_id'], dtype=np.uint64), thr_expected=thr.astype(np.uint8))
        if c['mask'] is not None:
            arrays['mask'] = c['mask']
        if c['channel'] is not None:
            arrays['channel'] = np.array(c['channel'], dtype=np.int64)
        np.savez_compressed(os.path.join(HERE, 'sigma_%s.npz' % c['name']), **arrays)
        index[c['name']] = dict(shape=list(c['inp'].shape), sigma=c['sigma'], channel=c['channel'],
                                block_shape=list(c['block_shape']), threshold=c['threshold'], mode=c['mode'],
                                mask=c['mask'] is not None, n_components=int(arrays['labels_canon'].max()),
                                n_labels=int(res['n_labels']))
        print(c['name'], index[c['name']])
    with open(os.path.join(HERE, 'index_sigma.json'), 'w') as fh:
        json.dump(index, fh, indent=1, sort_keys=True)


if __name__ == '__main__':
    main()
