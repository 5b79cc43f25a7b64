#!/opt/conda/bin/python3.9
"""Golden DIGESTS at the BASELINE block shapes, made by running the REFERENCE's own job functions.

Run only in the build container (needs /root/reference and the conda python with
scikit-image 0.18.3), after `make -C oracle` (the synthetic input comes from the oracle's C
generator, which tests/test_oracle_golden.py pins to oracle/synth.py):

    /opt/conda/bin/python3.9 tests/golden/make_golden_large.py [case ...]

The five reference stages run exactly as in make_golden.py (run_reference: block_components ->
merge_offsets -> block_faces -> merge_assignments -> write, the reference's code with numpy
1.26.4 / skimage 0.18.3, small local stand-ins for luigi / nifty / vigra / elf, h5py storage),
on the deterministic synthetic boundary map at the BASELINE geometries:

    c1_*     (125, 1250, 1250), block (50, 512, 512)  -- config 1 (27 blocks, edge blocks 25 / 226)
    c2_*     (512, 512, 512),   block (128, 128, 128) -- config 2
    b64_*    (128, 1024, 1024), block (64, 512, 512)  -- the block shape of configs 3-5

The volumes are too large to commit, so tests/golden/large_index.json holds the generator
parameters and the reference's artefacts: block values, offsets, n_labels, maxId, the pair count
and SHA-256 digests of the canonical labels, canonical LUT, the raw block-local (skimage) labels
and the sorted unique face pairs (oracle.digest: C-order little-endian bytes).
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as MG  # noqa: E402  (sets up the reference packages + stubs)
from oracle import oracle as O  # noqa: E402
from oracle.synth import ellipsoid_mask  # noqa: E402

CASES = {
    'c1_greater': dict(shape=(125, 1250, 1250), origin=(0, 0, 0), block_shape=(50, 512, 512), mode='greater'),
    'c1_less': dict(shape=(125, 1250, 1250), origin=(0, 0, 0), block_shape=(50, 512, 512), mode='less'),
    'c2_greater': dict(shape=(512, 512, 512), origin=(0, 0, 0), block_shape=(128, 128, 128), mode='greater'),
    'b64_greater': dict(shape=(128, 1024, 1024), origin=(64, 512, 0), block_shape=(64, 512, 512), mode='greater'),
    'b64_less': dict(shape=(128, 1024, 1024), origin=(64, 512, 0), block_shape=(64, 512, 512), mode='less'),
    'b64_mask_less': dict(shape=(128, 1024, 1024), origin=(64, 512, 0), block_shape=(64, 512, 512), mode='less',
                          mask=0.45),
}
THRESHOLD = 0.5


def case_input(c):
    q = O.boundary_map(c['shape'], origin=c['origin'], as_q=True, n_threads=8)
    inp = q.astype(np.float32) / np.float32(256)
    mask = ellipsoid_mask(c['shape'], c['mask']) if c.get('mask') else None
    return inp, mask


def main():
    names = sys.argv[1:] or list(CASES)
    path = os.path.join(HERE, 'large_index.json')
    index = json.load(open(path)) if os.path.exists(path) else {}
    for name in names:
        c = CASES[name]
        t = time.time()
        inp, mask = case_input(c)
        res = MG.run_reference(inp, c['block_shape'], THRESHOLD, c['mode'], mask=mask, n_jobs_bc=4,
                               n_jobs_bf=1, compression=None)
        del inp
        assert int(res['local_labels'].max()) < 2 ** 32
        entry = dict(shape=list(c['shape']), origin=list(c['origin']), block_shape=list(c['block_shape']),
                     threshold=THRESHOLD, mode=c['mode'], mask_semi_axes=c.get('mask'),
                     seed=0x5EED, generator='oracle.boundary_map (q / 256)',
                     block_values=[int(v) for v in res['block_values']],
                     offsets=[int(v) for v in res['offsets']],
                     empty_blocks=[int(v) for v in res['empty_blocks']],
                     n_labels=int(res['n_labels']), max_id=int(res['max_id']),
                     n_pairs=int(len(res['pairs'])),
                     digest_pairs=O.digest(res['pairs'].astype(np.uint64)),
                     digest_local_labels_u32=O.digest(res['local_labels'].astype(np.uint32)),
                     digest_labels_canon_u32=O.digest(O.canon_fast(res['labels'])),
                     digest_lut_canon_u32=O.digest(O.canon_fast(res['lut'])),
                     n_components=int(O.canon_fast(res['labels']).max()),
                     reference_seconds=round(time.time() - t, 1))
        index[name] = entry
        print(name, {k: v for k, v in entry.items() if k not in ('block_values', 'offsets', 'empty_blocks')},
              flush=True)
        with open(path, 'w') as fh:
            json.dump(index, fh, indent=1, sort_keys=True)


if __name__ == '__main__':
    main()
