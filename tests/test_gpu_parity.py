"""Parity of the HIP path with the oracle and with the reference's golden vectors.
All tests here run on an MI355X through the C ABI (libcc_mi355x.so)."""
import numpy as np
import pytest

from conftest import golden_index, load_golden
from oracle import oracle as O

pytestmark = pytest.mark.gpu
CASES = sorted(golden_index().items())
IDS = [c[0] for c in CASES]


def _quirk_jobs(meta):
    """max_jobs of the golden's block_faces run when it exercises the reference's empty-job
    branch (merge_assignments.py:115-123), else 0."""
    return meta['n_jobs_block_faces'] if meta['quirk'] else 0


def _check_against_oracle(ctx, inp, block_shape, thr, mode, mask=None, res=None, lab=None, quirk_jobs=0):
    if lab is None:
        ctx.set_empty_job_quirk(quirk_jobs)
        try:
            lab, res = ctx.label_volume(inp, block_shape, thr, mode, mask)
        finally:
            ctx.set_empty_job_quirk(0)
    r = O.label_volume(inp, block_shape, thr, mode, mask, n_threads=8, quirk_n_jobs=quirk_jobs)
    nb = len(r['values'])
    np.testing.assert_array_equal(lab, r['labels'])          # raw uint64, bit-exact
    np.testing.assert_array_equal(ctx.block_values(nb), r['values'])
    np.testing.assert_array_equal(ctx.offsets(nb), r['offsets'])
    assert res['n_labels'] == r['n_labels']
    assert res['max_id'] == r['max_id']
    np.testing.assert_array_equal(ctx.lut(res['n_labels']), r['lut'])
    return lab, res, r


@pytest.mark.parametrize('name,meta', CASES, ids=IDS)
def test_fused_path_golden(ctx, name, meta):
    d = load_golden(name)
    lab, res, r = _check_against_oracle(ctx, d['input'], meta['block_shape'], float(d['threshold']),
                                        meta['mode'], d.get('mask'), quirk_jobs=_quirk_jobs(meta))
    assert res['identity_lut'] == int(bool(meta['quirk']))
    # against the reference itself (canonical relabel = the parity contract)
    np.testing.assert_array_equal(O.canon(lab), d['labels_canon'])
    np.testing.assert_array_equal(ctx.block_values(len(d['block_values'])), d['block_values'])
    np.testing.assert_array_equal(ctx.offsets(len(d['offsets'])), d['offsets'])
    assert res['n_labels'] == int(d['n_labels'])
    assert res['max_id'] == int(d['max_id'])
    np.testing.assert_array_equal(O.canon(ctx.lut(res['n_labels'])), d['lut_canon'])
    assert res['n_components'] == int(d['labels_canon'].max())


@pytest.mark.parametrize('name,meta', CASES, ids=IDS)
def test_stage_level_golden(ctx, name, meta):
    """block_components -> merge_offsets -> block_faces -> merge_assignments -> write, one
    C-ABI entry per reference job, each artefact against the reference's."""
    import torch
    d = load_golden(name)
    x = torch.from_numpy(d['input']).cuda()
    m = torch.from_numpy(d['mask']).cuda() if 'mask' in d else None
    local, values = ctx.block_components(x, meta['block_shape'], float(d['threshold']), meta['mode'], m)
    np.testing.assert_array_equal(local.cpu().numpy().view(np.uint64), d['local_labels'].astype(np.uint64))
    np.testing.assert_array_equal(values, d['block_values'])
    from cluster_tools_amd import _lib
    offsets, empty, n_labels = _lib.merge_offsets(values)
    np.testing.assert_array_equal(offsets, d['offsets'])
    np.testing.assert_array_equal(empty, d['empty_blocks'])
    assert n_labels == int(d['n_labels'])
    pairs, flags = ctx.block_faces(local, meta['block_shape'], offsets, with_block_flags=True)
    np.testing.assert_array_equal(pairs, d['pairs'])
    from cluster_tools_amd.thresholded_components.merge_assignments import any_empty_job
    if meta['quirk']:
        # every block_faces job of the reference run must be checked: one without pairs -> identity
        assert any_empty_job(flags, _quirk_jobs(meta))
        lut = np.arange(n_labels, dtype=np.uint64)
    else:
        assert any_empty_job(flags, 1) == (len(pairs) == 0)     # one job: empty only without pairs
        lut = ctx.merge_assignments(pairs, n_labels)
    np.testing.assert_array_equal(O.canon(lut), d['lut_canon'])
    ctx.write(local, meta['block_shape'], offsets, lut)
    np.testing.assert_array_equal(O.canon(local.cpu().numpy()), d['labels_canon'])


def test_device_and_host_paths_agree(ctx):
    import torch
    d = load_golden('bmap_big_less')
    host, _ = ctx.label_volume(d['input'], (32, 64, 64), 0.5, 'less')
    dev, _ = ctx.label_volume(torch.from_numpy(d['input']).cuda(), (32, 64, 64), 0.5, 'less')
    np.testing.assert_array_equal(host, dev.cpu().numpy().view(np.uint64))


SYNTH = [
    ((64, 256, 256), (32, 128, 128), 'greater'),
    ((64, 256, 256), (32, 128, 128), 'less'),
    ((100, 300, 200), (50, 128, 100), 'less'),     # odd x extents, edge blocks
    ((96, 200, 250), (25, 64, 64), 'greater'),     # odd block z (partial cubes at block ends)
    ((70, 130, 190), (70, 130, 190), 'less'),      # one block, many tiles: 26-conn tile seams
    ((33, 65, 129), (11, 13, 43), 'greater'),      # tiles smaller than TX, odd everything
    ((128, 128, 128), (128, 128, 128), 'greater'),
]


@pytest.mark.parametrize('shape,bs,mode', SYNTH[:6])
def test_stage_path_vs_oracle(ctx, shape, bs, mode):
    """The stage entry points chained (block_components -> merge_offsets -> block_faces ->
    merge_assignments -> write; fused=False) on synthetic volumes larger than the goldens: face
    rows over several row groups of k_face_pairs, block rows changing inside a group, odd X (the
    8-B load path) and even X (16-B loads): final labels bit-exact against the oracle's."""
    import torch
    from cluster_tools_amd import _lib
    inp = O.boundary_map(shape, origin=(7, 3, 1))
    r = O.label_volume(inp, bs, 0.5, mode, None, n_threads=8)
    local, values = ctx.block_components(torch.from_numpy(inp).cuda(), bs, 0.5, mode)
    np.testing.assert_array_equal(values, r['values'])
    offsets, _, n_labels = _lib.merge_offsets(values)
    assert n_labels == r['n_labels']
    pairs = ctx.block_faces(local, bs, offsets)
    lut = ctx.merge_assignments(pairs, n_labels)
    np.testing.assert_array_equal(lut, r['lut'])
    ctx.write(local, bs, offsets, lut)
    np.testing.assert_array_equal(local.cpu().numpy().view(np.uint64), r['labels'])


@pytest.mark.parametrize('n_jobs', [1, 4, 27, 1000])
def test_empty_job_emulation_vs_oracle(ctx, n_jobs):
    """CC_OPT_EMPTY_JOB_QUIRK against the oracle's emulation for several max_jobs: the LUT is the
    identity exactly when one of the min(n_blocks, max_jobs) face jobs has no pair."""
    inp = O.boundary_map((40, 72, 88), origin=(5, 5, 5))
    for mode in ('greater', 'less'):
        _, res, r = _check_against_oracle(ctx, inp, (16, 32, 32), 0.5, mode, quirk_jobs=n_jobs)
        assert res['identity_lut'] == int(np.array_equal(r['lut'], np.arange(r['n_labels'])))


@pytest.mark.parametrize('shape,bs,mode', SYNTH)
def test_synthetic_vs_oracle(ctx, shape, bs, mode):
    inp = O.boundary_map(shape, origin=(7, 3, 1))
    _check_against_oracle(ctx, inp, bs, 0.5, mode)


@pytest.mark.parametrize('shape,bs,mode', SYNTH[:4])
def test_continuous_synthetic_vs_oracle(ctx, shape, bs, mode):
    """Continuous (dithered) input: the speculated intervals miss the exact ones."""
    inp = O.boundary_map(shape, origin=(7, 3, 1), dither=True)
    _check_against_oracle(ctx, inp, bs, 0.5, mode)
    _check_against_oracle(ctx, inp, bs, 0.37, mode)


@pytest.mark.parametrize('density', [0.2, 0.45, 0.6])
def test_white_noise_tile_seams(ctx, density):
    """White noise hits every 26-neighbour configuration at every tile seam."""
    rng = np.random.default_rng(int(density * 100))
    inp = rng.random((40, 80, 150), dtype=np.float32)
    _check_against_oracle(ctx, inp, (40, 80, 150), density, 'less')
    _check_against_oracle(ctx, inp, (20, 40, 75), 1 - density, 'greater')


def test_max_runs_per_tile(ctx):
    """Worst case for the tile union-find: every 2x2x2 cube occupied but no two x-neighbouring
    cubes linked (foreground only at even x), i.e. one run per cube (4096 per tile), plus
    white noise in the odd columns of a few slabs so some runs do link."""
    rng = np.random.default_rng(11)
    inp = np.zeros((48, 96, 192), dtype=np.float32)
    inp[:, :, 0::2] = 1.0
    inp[24:, :, 1::2] = (rng.random((24, 96, 96)) < 0.3).astype(np.float32)
    _check_against_oracle(ctx, inp, (48, 96, 192), 0.5, 'greater')
    _check_against_oracle(ctx, inp, (16, 32, 64), 0.5, 'greater')
    _check_against_oracle(ctx, inp, (48, 96, 192), 0.5, 'less')


@pytest.mark.parametrize('outlier', [-1.0, -1.0 / 32, 3.0, 1.0 + 1.0 / 64])
@pytest.mark.parametrize('mode,thr', [('greater', 0.5), ('less', 0.5), ('equal', 0.5), ('greater', 0.3)])
def test_speculated_interval_corrected(ctx, mode, thr, outlier):
    """Quantized data whose block extremes the sample misses (one outlier voxel off the sampled
    rows): the guessed interval is wrong; tiles with voxels between the guessed and the exact
    bounds must be relabelled (large outliers), the others kept (small outliers)."""
    rng = np.random.default_rng(3)
    inp = (rng.integers(0, 17, (64, 128, 192)) / np.float32(16)).astype(np.float32)
    inp[1, 1, 5] = outlier               # block (0, 0, 0); sample rows are z = 8 mod 16, y = 16 mod 32
    inp[33, 70, 100] = outlier           # block (1, 1, 1)
    for bs in [(32, 64, 96), (64, 128, 192)]:
        _, res, _ = _check_against_oracle(ctx, inp, bs, thr, mode)
        if mode != 'equal' and outlier in (-1.0, 3.0):
            assert res['n_relabelled_tiles'] > 0        # the guess moved past quantization levels
        if (mode, thr, outlier) == ('greater', 0.3, -1.0 / 32):
            assert res['n_relabelled_tiles'] == 0       # guess != exact, but no voxel in between
    mask = (rng.random(inp.shape) < 0.9).astype(np.uint8)
    _check_against_oracle(ctx, inp, (32, 64, 96), thr, mode, mask)


@pytest.mark.parametrize('mode', ['greater', 'less'])
@pytest.mark.parametrize('value', [-0.0, -1e-30, -0.25])
def test_sign_bit_values_off_sample(ctx, mode, value):
    """Values with the sign bit set (-0, a negative denormal, a negative number) off the sampled
    rows of otherwise non-negative data: the guessed interval and the block statistics must come
    out exact (statistics in the IEEE total order, -0 < +0), with and without a mask."""
    rng = np.random.default_rng(11)
    inp = (rng.integers(0, 17, (64, 128, 192)) / np.float32(16)).astype(np.float32)
    inp[1, 1, 5] = value                  # off the sampled rows (z = 8 mod 16, y = 16 mod 32)
    inp[40, 77, 130] = value
    inp[63, 127, 191] = value             # last voxel of the last (full) tile
    for bs in [(32, 64, 96), (64, 128, 192)]:
        _check_against_oracle(ctx, inp, bs, 0.5, mode)
    mask = (rng.random(inp.shape) < 0.9).astype(np.uint8)
    _check_against_oracle(ctx, inp, (32, 64, 96), 0.5, mode, mask)


def test_mask_vs_oracle(ctx):
    from oracle.synth import ellipsoid_mask
    shape = (64, 160, 192)
    inp = O.boundary_map(shape)
    mask = ellipsoid_mask(shape, 0.4)
    _check_against_oracle(ctx, inp, (32, 64, 64), 0.5, 'greater', mask)
    _check_against_oracle(ctx, inp, (32, 64, 64), 0.5, 'less', mask * 200)


def test_normalisation_edge_cases(ctx):
    rng = np.random.default_rng(5)
    x = rng.random((32, 48, 64), dtype=np.float32)
    x[:16, :24, :32] = x[:16, :24, :32] * np.float32(1e6) - np.float32(3e5)
    x[16:, 24:, 32:] = np.float32(-2.5)                       # constant block
    x[:16, 24:, 32:] = np.float32(np.nan)
    x[20, 5, 7] = np.float32(np.inf)
    x[3, 30, 3] = np.float32(-np.inf)
    x[16:, :24, :32] = (x[16:, :24, :32] * np.float32(1e-40)).astype(np.float32)   # denormals
    for mode, thr in [('greater', 0.5), ('less', 0.5), ('equal', 0.0), ('less', 0.1), ('greater', 1e-7)]:
        _check_against_oracle(ctx, x, (16, 24, 32), thr, mode)


def test_generator_matches_oracle(ctx):
    for shape, origin in [((40, 70, 300), (3, 5, 7)), ((17, 33, 513), (64, 0, 1000))]:
        g = ctx.generate_boundary_map(shape, origin=origin).cpu().numpy()
        np.testing.assert_array_equal(g, O.boundary_map(shape, origin=origin))
        g = ctx.generate_boundary_map(shape, origin=origin, dither=True).cpu().numpy()
        np.testing.assert_array_equal(g, O.boundary_map(shape, origin=origin, dither=True))


def test_repeat_runs_identical(ctx):
    import torch
    x = ctx.generate_boundary_map((128, 512, 512))
    a, ra = ctx.label_volume(x, (64, 256, 256), 0.5, 'less')
    b, rb = ctx.label_volume(x, (64, 256, 256), 0.5, 'less')
    assert torch.equal(a, b) and ra == rb


@pytest.mark.slow
def test_c2_vs_oracle(ctx):
    """BASELINE config 2 (512^3, block 128^3) bit-exact against the C oracle."""
    x = ctx.generate_boundary_map((512, 512, 512))
    lab, res = ctx.label_volume(x, (128, 128, 128), 0.5, 'greater')
    inp = x.cpu().numpy()
    _check_against_oracle(ctx, inp, (128, 128, 128), 0.5, 'greater', res=res,
                          lab=lab.cpu().numpy().view(np.uint64))


@pytest.mark.parametrize('shape,bs,mode', SYNTH[:5])
def test_global_stitch_fallback(ctx, shape, bs, mode):
    """Intra-block seams through the global union-find (the path for blocks whose pair lists or
    component counts exceed the per-block LDS union-find) give the same results."""
    inp = O.boundary_map(shape, origin=(7, 3, 1))
    ctx.set_debug(1)
    try:
        _check_against_oracle(ctx, inp, bs, 0.5, mode)
    finally:
        ctx.set_debug(0)


def test_white_noise_large_block(ctx):
    """Many components per tile and per block (block pair lists / LDS capacity overflow -> mixed
    LDS and global stitching within one volume)."""
    rng = np.random.default_rng(11)
    inp = rng.random((64, 192, 256), dtype=np.float32)
    _check_against_oracle(ctx, inp, (64, 192, 256), 0.3, 'less')
    _check_against_oracle(ctx, inp, (32, 96, 128), 0.3, 'less')


@pytest.mark.parametrize('kind', ['inter_overflow', 'block_lcap_overflow', 'both'])
def test_fallback_paths_structured(ctx, kind):
    """Patterns that overflow the LDS lists by construction, so the launch-only-when-flagged
    fallbacks (k_stitch<false> when a block exceeds the LDS union-find, k_stitch<true> when a
    tile's block-face pair list overflows) run next to the LDS paths of other blocks / tiles:
      inter_overflow: 2-voxel columns on a 2-lattice across each z block face (512 distinct
        6-connected pairs per tile face > 256 slots);
      block_lcap_overflow: isolated voxels on a 2-lattice in the first block only (16 k
        components > 8 k LDS slots), ordinary data elsewhere."""
    shape, bs = (64, 128, 256), (16, 64, 128)
    base = O.boundary_map(shape, origin=(1, 2, 3))
    inp = np.ones(shape, dtype=np.float32)
    z, y, x = np.meshgrid(np.arange(shape[0]), np.arange(shape[1]), np.arange(shape[2]), indexing='ij')
    lat = (y % 2 == 0) & (x % 2 == 0)
    if kind in ('inter_overflow', 'both'):
        face = (z % bs[0] == 0) | (z % bs[0] == bs[0] - 1)        # the two voxel planes at each z block face
        inp[face & lat] = 0.0
    if kind in ('block_lcap_overflow', 'both'):
        first = (z < bs[0]) & (y < bs[1]) & (x < bs[2])
        inp[first] = 1.0
        inp[first & lat & (z % 2 == 0)] = 0.0
        inp[~first & (z >= 2 * bs[0])] = base[~first & (z >= 2 * bs[0])]
    _check_against_oracle(ctx, inp, bs, 0.5, 'less')


def _full_size_vs_oracle(ctx, shape, bs, mode, masked=False, dither=False):
    """The fused path on the device against the C oracle on the same synthetic volume, at a
    BASELINE size: raw uint64 labels compared on the device, block values / offsets / n_labels /
    maxId / LUT on the host."""
    import os
    import torch
    x = ctx.generate_boundary_map(shape, dither=dither)
    mask = None
    if masked:
        from cluster_tools_amd.synthetic import ellipsoid_mask_device
        mask = ellipsoid_mask_device(shape, 0, shape[0], x.device)
        torch.cuda.synchronize()
    lab, res = ctx.label_volume(x, bs, 0.5, mode, mask=mask)
    inp = x.cpu().numpy()
    hmask = None if mask is None else mask.cpu().numpy()
    del x, mask
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    r = O.label_volume(inp, bs, 0.5, mode, hmask, n_threads=threads)
    del inp, hmask
    assert res['n_labels'] == r['n_labels'] and res['max_id'] == r['max_id']
    nb = len(r['values'])
    np.testing.assert_array_equal(ctx.block_values(nb), r['values'])
    np.testing.assert_array_equal(ctx.offsets(nb), r['offsets'])
    np.testing.assert_array_equal(ctx.lut(res['n_labels']), r['lut'])
    ref = torch.from_numpy(r.pop('labels').view(np.int64)).cuda()
    assert bool(torch.equal(lab, ref))
    del ref, lab
    torch.cuda.empty_cache()
    return res


@pytest.mark.slow
@pytest.mark.parametrize('mode', ['greater', 'less'])
def test_c3_vs_oracle(ctx, mode):
    """BASELINE config 3 (1024 x 2048 x 2048, block 64 x 512 x 512) bit-exact against the C oracle:
    'greater' is the benchmarked workload (one giant membrane component: union-find contention),
    'less' the 150 k-component case (where a tile-CCL race once moved small pieces)."""
    _full_size_vs_oracle(ctx, (1024, 2048, 2048), (64, 512, 512), mode)


@pytest.mark.slow
@pytest.mark.parametrize('mode', ['greater', 'less'])
def test_c3_mask_vs_oracle(ctx, mode):
    """C3 + the ellipsoid uint8 mask (config 4's input, here as one volume) bit-exact against the
    C oracle (block_components.py:185-233: mask ANDed after the threshold, empty blocks skipped)."""
    _full_size_vs_oracle(ctx, (1024, 2048, 2048), (64, 512, 512), mode, masked=True)


@pytest.mark.slow
@pytest.mark.parametrize('mode', ['greater', 'less'])
def test_c1_shape_vs_oracle(ctx, mode):
    """BASELINE config 1's geometry (CREMI-sized 125 x 1250 x 1250, the reference default block
    50 x 512 x 512: 27 blocks, edge blocks 25 / 226 wide) bit-exact against the C oracle."""
    res = _full_size_vs_oracle(ctx, (125, 1250, 1250), (50, 512, 512), mode)
    assert res['n_blocks'] == 27


@pytest.mark.slow
@pytest.mark.parametrize('mode', ['greater', 'less'])
def test_c3_continuous_vs_oracle(ctx, mode):
    """C3 on continuous (dithered, non-quantized) float32 input: the speculative front's guessed
    intervals are not exact here, so k_fix relabels the tiles with voxels between the guessed
    and exact bounds; the result must still be bit-exact."""
    res = _full_size_vs_oracle(ctx, (1024, 2048, 2048), (64, 512, 512), mode, dither=True)
    assert res['n_relabelled_tiles'] < 131072 // 4


@pytest.mark.slow
@pytest.mark.parametrize('mode', ['greater'])
def test_c5_slab_vs_oracle(ctx, mode):
    """BASELINE config 5's per-rank slab: (256, 4096, 4096), block (64, 512, 512) -- 4096-voxel rows
    (32 KB apart), the geometry on which the host picks k_pass2's z-fastest tile order (X >= 4096)
    -- bit-exact against the C oracle (same voxel count as C3)."""
    _full_size_vs_oracle(ctx, (256, 4096, 4096), (64, 512, 512), mode)


PASS2_ORDER_CASES = [
    ((96, 320, 448), (32, 128, 128), 'greater'),
    ((96, 320, 448), (32, 128, 128), 'less'),
    ((70, 130, 300), (35, 65, 150), 'less'),       # odd blocks: partial tiles at every block end
]


@pytest.mark.parametrize('order', ['0', '1', '2'])
@pytest.mark.parametrize('shape,bs,mode', PASS2_ORDER_CASES)
def test_pass2_tile_order_vs_oracle(ctx, monkeypatch, shape, bs, mode, order):
    """Every k_pass2 tile order (x fastest / z fastest / XCD-contiguous; CC_PASS2_ORDER, read on
    every call) on the fused path gives the oracle's labels (order 1 was only reached
    by X >= 4096; order 2 otherwise only by rows that are not 128-B aligned)."""
    monkeypatch.setenv('CC_PASS2_ORDER', order)
    inp = O.boundary_map(shape, origin=(5, 9, 2))
    _check_against_oracle(ctx, inp, bs, 0.5, mode)
    inp = O.boundary_map(shape, origin=(5, 9, 2), dither=True)
    _check_against_oracle(ctx, inp, bs, 0.41, mode)


UNALIGNED_CASES = [
    ((40, 72, 258), (32, 64, 130)),      # X = 2 mod 4
    ((36, 70, 322), (36, 70, 322)),
    ((33, 66, 195), (33, 66, 195)),      # odd X
]


@pytest.mark.parametrize('mode', ['greater', 'less'])
@pytest.mark.parametrize('shape,bs', UNALIGNED_CASES)
def test_unaligned_rows_vs_oracle(ctx, shape, bs, mode):
    """Rows that are not 16-B aligned (X % 4 != 0, as C1's 1250): k_spec's lane = x path on full
    tiles and the XCD-contiguous tile order of k_spec / k_pass2; quantized, masked and continuous
    input."""
    rng = np.random.default_rng(11)
    inp = O.boundary_map(shape, origin=(3, 7, 1))
    _check_against_oracle(ctx, inp, bs, 0.5, mode)
    mask = (rng.random(shape) < 0.9).astype(np.uint8)
    _check_against_oracle(ctx, inp, bs, 0.5, mode, mask)
    inp = O.boundary_map(shape, origin=(3, 7, 1), dither=True)
    _check_against_oracle(ctx, inp, bs, 0.41, mode)


@pytest.mark.parametrize('mshape,shape', [((20, 36, 44), (40, 72, 88)), ((40, 72, 88), (40, 72, 88)),
                                          ((13, 50, 17), (40, 72, 88)), ((80, 30, 200), (40, 72, 89)),
                                          # X % 16 == 0: the 16-byte-per-thread kernel
                                          ((20, 36, 48), (40, 72, 96)), ((13, 50, 1000), (24, 40, 2048))])
def test_resized_mask_device_vs_oracle(ctx, mshape, shape):
    """cc_resize_mask_nearest (elf ResizedVolume(order=0) stand-in, volume_utils.py:174-184) against
    the oracle's rule, whole volume and z-slabs; then the labelling with it (parity with elf
    itself unpinned: elf is absent)."""
    rng = np.random.default_rng(sum(mshape))
    m = (rng.random(mshape) < 0.6).astype(np.uint8) * 3
    want = O.resize_mask_nearest(m, shape)
    np.testing.assert_array_equal(ctx.resize_mask(m, shape).cpu().numpy(), want)
    np.testing.assert_array_equal(ctx.resize_mask(m, shape, z0=7, nz=16).cpu().numpy(), want[7:23])
    inp = O.boundary_map(shape, origin=(2, 3, 4))
    _check_against_oracle(ctx, inp, (16, 32, 32), 0.5, 'less', want)


@pytest.mark.parametrize('fast', ['0', '1'])
@pytest.mark.parametrize('shape,bs,mode', SYNTH[:4])
def test_both_schedules_vs_oracle(ctx, monkeypatch, fast, shape, bs, mode):
    """The one-read-back schedule (default: every count stays on the device, one read-back per
    run) and the host-synchronised schedule (CC_FAST=0) give the oracle's labels, quantized and
    continuous input (the device-gated k_fix path)."""
    monkeypatch.setenv('CC_FAST', fast)
    x = O.boundary_map(shape, origin=(2, 5, 1))
    _check_against_oracle(ctx, x, bs, 0.5, mode)
    xc = O.boundary_map(shape, origin=(2, 5, 1), dither=True)
    _check_against_oracle(ctx, xc, bs, 0.5, mode)


def test_root_capacity_redo(monkeypatch):
    """More block-local roots than a context's root arrays hold (CC_ROOT_CAP: the first capacity):
    the one read-back carries RF_ROOTS, the run is redone host-synchronised (two block scans)
    with the oracle's result, and the capacity is raised so the next run needs one pass."""
    from cluster_tools_amd import _lib
    monkeypatch.setenv('CC_ROOT_CAP', '8')
    shape, bs = (64, 96, 160), (32, 48, 64)
    x = O.boundary_map(shape, origin=(0, 3, 7))
    with _lib.Context(0) as c:
        c.set_profiling(1)
        for passes in (2, 1):
            c.reset_profile()
            _check_against_oracle(c, x, bs, 0.5, 'less')
            prof = c.profile()         # the one-read-back pass scans in k_scan_emit, the redo in k_block_scan
            assert sum(prof.get(k, {}).get('count', 0) for k in ('k_block_scan', 'k_scan_emit')) == passes


def test_empty_tiles_context_reuse(ctx):
    """Tiles without foreground store no bit rows and zero faces: one context labels inputs whose
    empty tiles move (non-empty -> empty -> non-empty), with and without a mask and through a
    speculation miss (the k_fix path re-runs pass 1 of such tiles), always equal to the oracle --
    nothing of an earlier run leaks through the skipped stores."""
    shape, bs = (64, 160, 256), (32, 64, 128)
    base = O.boundary_map(shape, origin=(2, 7, 3))
    a = base.copy()
    a[:, :, 128:] = 0.0                    # x half empty ('greater')
    b = base.copy()
    b[:, :80, :] = 0.0                     # y half empty instead
    c = base.copy()
    c[5, 9, 200] = -3.0                    # an extreme off the sampled rows: k_fix relabels tiles
    c[:32] = 0.0
    for inp in (base, a, b, a, c, base):
        _check_against_oracle(ctx, inp, bs, 0.5, 'greater')
        _check_against_oracle(ctx, inp, bs, 0.5, 'less')
    from oracle.synth import ellipsoid_mask
    m = ellipsoid_mask(shape)
    for inp in (base, b, base):
        _check_against_oracle(ctx, inp, bs, 0.5, 'greater', m)
