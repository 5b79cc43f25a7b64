"""The oracle (oracle/cc_oracle.c) against the golden vectors made by the reference's own
job functions (tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest

from conftest import golden_index, load_golden
from oracle import oracle as O

CASES = sorted(golden_index().items())


@pytest.mark.parametrize('name,meta', CASES, ids=[c[0] for c in CASES])
def test_oracle_matches_reference(name, meta):
    d = load_golden(name)
    quirk = meta['n_jobs_block_faces'] if meta['quirk'] else 0
    r = O.label_volume(d['input'], meta['block_shape'], float(d['threshold']), meta['mode'],
                       d.get('mask'), n_threads=3, quirk_n_jobs=quirk, want_local=True)
    # stage 1: skimage numbering of block-local components, bit-exact
    np.testing.assert_array_equal(r['local'], d['local_labels'].astype(np.uint64))
    # stage 2: merge_offsets artefacts, bit-exact
    np.testing.assert_array_equal(r['values'], d['block_values'])
    np.testing.assert_array_equal(r['offsets'], d['offsets'])
    np.testing.assert_array_equal(r['empty_blocks'], d['empty_blocks'])
    assert r['n_labels'] == int(d['n_labels'])
    # stage 3: face pairs, bit-exact
    pairs = O.face_pairs(r['local'], meta['block_shape'], r['offsets'], r['empty_blocks'])
    np.testing.assert_array_equal(pairs, d['pairs'])
    # stages 4-5: partition (canonical relabel) and maxId
    np.testing.assert_array_equal(O.canon(r['lut']), d['lut_canon'])
    np.testing.assert_array_equal(O.canon(r['labels']), d['labels_canon'])
    assert r['max_id'] == int(d['max_id']) == r['n_labels'] - 1


@pytest.mark.parametrize('name,meta', [c for c in CASES if not c[1]['quirk'] and not c[1]['mask']],
                         ids=[c[0] for c in CASES if not c[1]['quirk'] and not c[1]['mask']])
def test_graph_definition_matches_reference(name, meta):
    """Independent restatement: 26-conn inside blocks, 6-conn across."""
    d = load_golden(name)
    fg = d['labels_canon'] != 0
    np.testing.assert_array_equal(O.graph_components(fg, meta['block_shape']), d['labels_canon'])


def test_quirk_differs_from_intended():
    d = load_golden('bmap_quirk')
    e = load_golden('bmap_greater')
    assert d['labels_canon'].max() > e['labels_canon'].max()


def test_generator_c_matches_numpy():
    from oracle.synth import boundary_map
    for shape, origin in [((20, 37, 50), (0, 0, 0)), ((9, 40, 70), (31, 63, 95))]:
        np.testing.assert_array_equal(O.boundary_map(shape, origin, n_threads=2), boundary_map(shape, origin))
        d = O.boundary_map(shape, origin, n_threads=2, dither=True)
        np.testing.assert_array_equal(d, boundary_map(shape, origin, dither=True))
        # the dither stays below one quantization step and does not move q
        q = O.boundary_map(shape, origin, n_threads=2)
        assert np.all((d >= q) & (d < q + np.float32(1 / 256)))


def test_oracle_threads_invariant():
    x = O.boundary_map((40, 80, 96), n_threads=4)
    a = O.label_volume(x, (16, 32, 32), 0.5, 'less', n_threads=1)
    b = O.label_volume(x, (16, 32, 32), 0.5, 'less', n_threads=5)
    np.testing.assert_array_equal(a['labels'], b['labels'])
    np.testing.assert_array_equal(a['lut'], b['lut'])
