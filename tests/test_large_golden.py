"""Parity at the BASELINE block shapes against the REFERENCE's own output.

tests/golden/large_index.json holds what the reference's five job functions produced
(tests/golden/make_golden_large.py: block_components -> merge_offsets -> block_faces ->
merge_assignments -> write, scikit-image 0.18.3) on the synthetic boundary map at the geometries
of BASELINE configs 1 and 2 and at the (64, 512, 512) block of configs 3-5: block values, offsets,
n_labels, maxId, and SHA-256 digests of the canonical labels / LUT, the raw skimage block-local
labels and the sorted unique face pairs.  The volumes are regenerated from the generator
parameters (oracle.boundary_map, pinned to oracle/synth.py by test_oracle_golden.py).

CPU tests pin the C oracle to these digests; GPU tests check the HIP path -- fused and stage by
stage through the C ABI -- against the same digests directly."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import oracle as O


def _index():
    with open(os.path.join(GOLDEN, 'large_index.json')) as f:
        return json.load(f)


CASES = sorted(_index().items())
IDS = [c[0] for c in CASES]


def _input(meta):
    from oracle.synth import ellipsoid_mask
    q = O.boundary_map(meta['shape'], origin=meta['origin'], seed=meta['seed'], as_q=True, n_threads=8)
    inp = q.astype(np.float32) / np.float32(256)
    mask = ellipsoid_mask(tuple(meta['shape']), meta['mask_semi_axes']) if meta['mask_semi_axes'] else None
    return inp, mask


def _check_small(meta, values, offsets, n_labels, max_id):
    np.testing.assert_array_equal(np.asarray(values, dtype=np.uint64), np.array(meta['block_values'], dtype=np.uint64))
    np.testing.assert_array_equal(np.asarray(offsets, dtype=np.uint64), np.array(meta['offsets'], dtype=np.uint64))
    assert int(n_labels) == meta['n_labels'] and int(max_id) == meta['max_id']


@pytest.mark.slow
@pytest.mark.parametrize('name,meta', CASES, ids=IDS)
def test_oracle_vs_reference_digests(name, meta):
    inp, mask = _input(meta)
    r = O.label_volume(inp, meta['block_shape'], meta['threshold'], meta['mode'], mask,
                       n_threads=8, want_local=True)
    _check_small(meta, r['values'], r['offsets'], r['n_labels'], r['max_id'])
    assert O.digest(r['local'].astype(np.uint32)) == meta['digest_local_labels_u32']
    assert O.digest(O.canon_fast(r['labels'])) == meta['digest_labels_canon_u32']
    assert O.digest(O.canon_fast(r['lut'])) == meta['digest_lut_canon_u32']


@pytest.mark.gpu
@pytest.mark.parametrize('name,meta', CASES, ids=IDS)
def test_fused_vs_reference_digests(ctx, name, meta):
    import torch
    inp, mask = _input(meta)
    x = torch.from_numpy(inp).cuda()
    m = None if mask is None else torch.from_numpy(mask).cuda()
    lab, res = ctx.label_volume(x, meta['block_shape'], meta['threshold'], meta['mode'], mask=m)
    nb = len(meta['block_values'])
    _check_small(meta, ctx.block_values(nb), ctx.offsets(nb), res['n_labels'], res['max_id'])
    assert O.digest(O.canon_fast(lab.cpu().numpy())) == meta['digest_labels_canon_u32']
    assert O.digest(O.canon_fast(ctx.lut(res['n_labels']))) == meta['digest_lut_canon_u32']
    assert res['n_components'] == meta['n_components']


@pytest.mark.gpu
@pytest.mark.parametrize('name,meta', CASES, ids=IDS)
def test_stages_vs_reference_digests(ctx, name, meta):
    """One C-ABI call per reference job (cc_block_components, cc_merge_offsets, cc_block_faces,
    cc_merge_assignments, cc_write), each artefact against the reference's."""
    import torch
    from cluster_tools_amd import _lib
    inp, mask = _input(meta)
    x = torch.from_numpy(inp).cuda()
    m = None if mask is None else torch.from_numpy(mask).cuda()
    bs = meta['block_shape']
    local, values = ctx.block_components(x, bs, meta['threshold'], meta['mode'], m)
    del x, m
    assert O.digest(local.cpu().numpy().astype(np.uint32)) == meta['digest_local_labels_u32']
    offsets, empty, n_labels = _lib.merge_offsets(values)
    _check_small(meta, values, offsets, n_labels, n_labels - 1)
    np.testing.assert_array_equal(empty, meta['empty_blocks'])
    pairs = ctx.block_faces(local, bs, offsets)
    assert len(pairs) == meta['n_pairs'] and O.digest(pairs) == meta['digest_pairs']
    lut = ctx.merge_assignments(pairs, n_labels)
    assert O.digest(O.canon_fast(lut)) == meta['digest_lut_canon_u32']
    ctx.write(local, bs, offsets, lut)
    assert O.digest(O.canon_fast(local.cpu().numpy())) == meta['digest_labels_canon_u32']
