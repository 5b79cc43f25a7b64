"""ctypes front-end of the CPU oracle (oracle/cc_oracle.c).

TEST INFRASTRUCTURE ONLY.  The oracle is the checker and the CPU baseline; only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import it.
The product (cluster_tools_amd) never imports anything from oracle/.

Build: `make -C oracle` (also done by __graft_entry__.build()).
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# override: the sanitizer build (tools/asan.sh) only
_LIB_PATH = os.environ.get('CC_ORACLE_LIB') or os.path.join(_HERE, 'libcc_oracle.so')
_lib = None

MODES = {'greater': 0, 'less': 1, 'equal': 2}


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            raise RuntimeError('oracle library missing: run `make -C oracle`')
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        i64 = ctypes.c_int64
        L.oracle_boundary_map.argtypes = [P, P, i64, i64, i64, i64, i64, i64, ctypes.c_uint64, ctypes.c_int,
                                          ctypes.c_int]
        L.oracle_boundary_map.restype = None
        L.oracle_label_volume.argtypes = [P, P, P, P, ctypes.c_double, ctypes.c_int, ctypes.c_int,
                                          P, P, P, P, P, P, i64, P, ctypes.c_int, P]
        L.oracle_label_volume.restype = ctypes.c_int
        L.oracle_n_blocks.argtypes = [P, P]
        L.oracle_n_blocks.restype = i64
        L.oracle_canon_u64.argtypes = [P, i64, P]
        L.oracle_canon_u64.restype = i64
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data


def boundary_map(shape, origin=(0, 0, 0), seed=0x5EED, n_threads=8, as_q=False, dither=False):
    """Synthetic boundary map (oracle/synth.py definition), float32 or uint8 q; dither: the
    continuous variant (q * 2^16 + 16-bit dither) / 2^24."""
    shape = tuple(int(s) for s in shape)
    out = np.empty(shape, dtype=np.uint8 if as_q else np.float32)
    args = (None, out) if as_q else (out, None)
    lib().oracle_boundary_map(_ptr(args[0]), _ptr(args[1]), *shape, *[int(o) for o in origin],
                              ctypes.c_uint64(seed), int(n_threads), int(bool(dither)))
    return out


def n_blocks(shape, block_shape):
    s = np.ascontiguousarray(shape, dtype=np.int64)
    b = np.ascontiguousarray(block_shape, dtype=np.int64)
    return int(lib().oracle_n_blocks(_ptr(s), _ptr(b)))


def label_volume(inp, block_shape, threshold, mode='greater', mask=None, n_threads=1,
                 quirk_n_jobs=0, want_local=False, want_lut=True):
    """Run the restated reference path.  Returns a dict of artefacts:
    labels (final uint64), values (n_i+1 or 0), offsets, n_labels, lut, max_id,
    empty_blocks, stage_seconds, and local (block-local labels) if want_local."""
    inp = np.ascontiguousarray(inp, dtype=np.float32)
    assert inp.ndim == 3
    if mask is not None:
        mask = np.ascontiguousarray(mask, dtype=np.uint8)
        assert mask.shape == inp.shape
    shape = np.array(inp.shape, dtype=np.int64)
    bs = np.array(block_shape, dtype=np.int64)
    nb = n_blocks(shape, bs)
    labels = np.empty(inp.shape, dtype=np.uint64)
    local = np.empty(inp.shape, dtype=np.uint64) if want_local else None
    values = np.empty(nb, dtype=np.uint64)
    offsets = np.empty(nb, dtype=np.uint64)
    n_labels = np.zeros(1, dtype=np.uint64)
    max_id = np.zeros(1, dtype=np.uint64)
    stage_s = np.zeros(5, dtype=np.float64)
    # n_labels <= n_blocks + voxels/1 ; size the LUT after a first cheap bound
    lut_cap = int(inp.size + nb + 1) if want_lut else 0
    lut = np.empty(lut_cap, dtype=np.uint64) if want_lut else None
    rc = lib().oracle_label_volume(_ptr(inp), _ptr(mask), _ptr(shape), _ptr(bs), float(threshold),
                                   MODES[mode], int(n_threads), _ptr(labels), _ptr(local),
                                   _ptr(values), _ptr(offsets), _ptr(n_labels), _ptr(lut),
                                   lut_cap, _ptr(max_id), int(quirk_n_jobs), _ptr(stage_s))
    if rc != 0:
        raise RuntimeError('oracle_label_volume failed: %d' % rc)
    nl = int(n_labels[0])
    out = dict(labels=labels, values=values, offsets=offsets, n_labels=nl,
               lut=None if lut is None else lut[:nl].copy(), max_id=int(max_id[0]),
               empty_blocks=np.nonzero(values == 0)[0], stage_seconds=stage_s)
    if want_local:
        out['local'] = local
    return out


def canon(labels):
    """First-occurrence (C order) consecutive relabel; 0 stays 0 (parity contract)."""
    flat = np.asarray(labels).ravel()
    out = np.zeros(flat.shape, dtype=np.uint32)
    nz = flat != 0
    if nz.any():
        vals = flat[nz]
        uniq, first, inv = np.unique(vals, return_index=True, return_inverse=True)
        order = np.argsort(first, kind='stable')
        rank = np.empty(len(uniq), dtype=np.uint32)
        rank[order] = np.arange(1, len(uniq) + 1, dtype=np.uint32)
        out[nz] = rank[inv.ravel()]
    return out.reshape(np.shape(labels))


def resize_mask_nearest(mask, shape):
    """A mask of another shape resized to `shape` by pixel-centre nearest neighbour, the rule
    cc_resize_mask_nearest implements for elf ResizedVolume(order=0) (volume_utils.py:174-184):
    src(c) = floor((c + 0.5) * m / S) per axis, result uint8 0 / 1.  (elf is absent: this restates
    the product's documented rule, parity with elf unpinned.)"""
    mask = np.asarray(mask)
    idx = []
    for m, S in zip(mask.shape, shape):
        c = np.arange(S, dtype=np.int64)
        idx.append(np.minimum(((2 * c + 1) * m) // (2 * S), m - 1))
    return (mask[np.ix_(*idx)] != 0).astype(np.uint8)


def canon_fast(labels):
    """canon() for large uint64 volumes (cc_oracle.c oracle_canon_u64: one pass, hash map)."""
    a = np.ascontiguousarray(labels)
    assert a.dtype.itemsize == 8
    a = a.view(np.uint64)
    out = np.empty(a.shape, dtype=np.uint32)
    if lib().oracle_canon_u64(_ptr(a), a.size, _ptr(out)) < 0:
        raise RuntimeError('oracle_canon_u64 failed')
    return out


def digest(a):
    """SHA-256 hex of an array's C-order little-endian bytes (golden digests of large cases)."""
    import hashlib
    a = np.ascontiguousarray(a)
    h = hashlib.sha256()
    flat = a.reshape(-1).view(np.uint8)
    step = 1 << 28
    for i in range(0, flat.size, step):
        h.update(flat[i:i + step].data)
    return h.hexdigest()


def face_pairs(local, block_shape, offsets, empty):
    """Deduplicated (K,2) face pairs of block_faces.py:87-137 from block-local labels."""
    shape = local.shape
    nbz, nby, nbx = [-(-s // b) for s, b in zip(shape, block_shape)]
    empty = set(int(e) for e in empty)
    out = []
    for b in range(nbz * nby * nbx):
        if b in empty:
            continue
        c = np.unravel_index(b, (nbz, nby, nbx))
        beg = [ci * bs for ci, bs in zip(c, block_shape)]
        end = [min(bg + bs, s) for bg, bs, s in zip(beg, block_shape, shape)]
        for axis in range(3):
            cn = list(c)
            cn[axis] += 1
            if cn[axis] >= (nbz, nby, nbx)[axis]:
                continue
            nb = int(np.ravel_multi_index(cn, (nbz, nby, nbx)))
            if nb in empty:
                continue
            sa = tuple(slice(bg, e) if d != axis else slice(e - 1, e)
                       for d, (bg, e) in enumerate(zip(beg, end)))
            sb = tuple(slice(bg, e) if d != axis else slice(e, e + 1)
                       for d, (bg, e) in enumerate(zip(beg, end)))
            la, lb = local[sa].ravel(), local[sb].ravel()
            keep = (la != 0) & (lb != 0)
            if keep.any():
                out.append(np.stack([la[keep] + offsets[b], lb[keep] + offsets[nb]], axis=1))
    if not out:
        return np.zeros((0, 2), dtype=np.uint64)
    return np.unique(np.concatenate(out, axis=0).astype(np.uint64), axis=0)


def graph_components(inp_fg, block_shape):
    """Independent restatement of the partition, via scipy:
    26-connectivity inside blocks, 6-connectivity across block faces.  Returns
    canonical labels.  Small inputs only."""
    from scipy.sparse import coo_matrix
    from scipy.sparse.csgraph import connected_components
    fg = np.asarray(inp_fg, dtype=bool)
    shape = fg.shape
    idx = np.arange(fg.size).reshape(shape)
    blk = [np.arange(s) // b for s, b in zip(shape, block_shape)]
    rows, cols = [], []
    for dz in (-1, 0, 1):
        for dy in (-1, 0, 1):
            for dx in (-1, 0, 1):
                if (dz, dy, dx) <= (0, 0, 0):
                    continue
                d = (dz, dy, dx)
                sl_a = tuple(slice(max(0, -o), s - max(0, o)) for o, s in zip(d, shape))
                sl_b = tuple(slice(a.start + o, a.stop + o) for a, o in zip(sl_a, d))
                ok = fg[sl_a] & fg[sl_b]
                n_axes = sum(1 for o in d if o != 0)
                same = np.ones(ok.shape, dtype=bool)
                for ax, o in enumerate(d):
                    if o == 0:
                        continue
                    ba = blk[ax][sl_a[ax]]
                    bb = blk[ax][sl_b[ax]]
                    shp = [1, 1, 1]
                    shp[ax] = -1
                    same &= (ba == bb).reshape(shp)
                allowed = same if n_axes > 1 else np.ones_like(same)
                ok &= allowed
                rows.append(idx[sl_a][ok])
                cols.append(idx[sl_b][ok])
    r = np.concatenate(rows)
    c = np.concatenate(cols)
    n = fg.size
    g = coo_matrix((np.ones(len(r), dtype=np.int8), (r, c)), shape=(n, n))
    _, lab = connected_components(g, directed=False)
    lab = (lab + 1).reshape(shape).astype(np.uint64)
    lab[~fg] = 0
    return canon(lab)


def threshold_volume(inp, block_shape, threshold, mode='greater'):
    """Threshold task restated in numpy (TEST INFRASTRUCTURE ONLY).

    Per block of the C-order block grid (nifty blocking from the origin, edge blocks truncated):
    normalize as cluster_tools/utils/volume_utils.py:98-105 (float32: subtract the min, divide
    by the max when it is > 0) and compare with the threshold as threshold.py:160-167 (python
    float against a float32 array: a float32 compare), stored as uint8 (threshold.py:170).
    """
    x = np.asarray(inp)
    out = np.zeros(x.shape, dtype=np.uint8)
    thr = np.float32(threshold)
    grids = [range(0, s, b) for s, b in zip(x.shape, block_shape)]
    with np.errstate(invalid='ignore', divide='ignore'):
        for z0 in grids[0]:
            for y0 in grids[1]:
                for x0 in grids[2]:
                    bb = (slice(z0, z0 + block_shape[0]), slice(y0, y0 + block_shape[1]),
                          slice(x0, x0 + block_shape[2]))
                    y = x[bb].astype(np.float32)
                    y -= y.min()
                    m = y.max()
                    if m > 0:
                        y /= m
                    if mode == 'greater':
                        r = y > thr
                    elif mode == 'less':
                        r = y < thr
                    elif mode == 'equal':
                        r = y == thr
                    else:
                        raise RuntimeError('Thresholding Mode %s not supported' % mode)
                    out[bb] = r.astype(np.uint8)
    return out


def channel_mean(inp4, channel):
    """Multi-channel input restated (TEST INFRASTRUCTURE ONLY): the selected channels of a
    (C, Z, Y, X) array averaged as block_components.py:150-159 / threshold.py:139-148 do it --
    np.mean(axis=0) of a stack in the dataset's dtype.  numpy reduces over the outer axis
    element by element in channel-list order (sum_0 = x_c0, sum_k = sum_{k-1} + x_ck), in float32
    for float32 input and in float64 for integer / float64 input, then divides by the channel
    count in that type; vu.normalize (volume_utils.py:99) casts the mean to float32 after.
    Written as explicit loops so the order is stated, not inherited from np.mean."""
    x = np.asarray(inp4)
    chans = [channel] if isinstance(channel, (int, np.integer)) else [int(c) for c in channel]
    acc_t = np.float32 if x.dtype == np.float32 else np.float64
    acc = x[chans[0]].astype(acc_t)
    for c in chans[1:]:
        acc = (acc + x[c].astype(acc_t)).astype(acc_t)
    acc = (acc / acc_t(len(chans))).astype(acc_t)
    return acc.astype(np.float32)


def gaussian_taps(sigma):
    """vigra Kernel1D<float>::initGaussian(sigma, 1.0) restated (TEST INFRASTRUCTURE ONLY; the
    reference's sigma_prefilter filter when fastfilters is absent, volume_utils.py:13-18,80-94;
    vigra is absent here, so this restatement is UNPINNED against vigra itself): radius
    (int)(3 sigma + 0.5) (at least 1); tap(x) = norm * expf(x*x * sigma2) for x = -r..r in float32,
    sigma2 = -0.5f / s / s, norm = float(1 / (sqrt(2 pi) * s)); then every tap times 1 / (sum of
    the taps, float32 left to right).  expf is libm's (the same function the library's host code
    calls).  Returns (taps float32[2r + 1], r)."""
    import ctypes
    import math
    libm = ctypes.CDLL('libm.so.6')
    expf = libm.expf
    expf.restype, expf.argtypes = ctypes.c_float, [ctypes.c_float]
    f32 = np.float32
    radius = max(1, int(3.0 * sigma + 0.5))
    s = f32(sigma)
    sigma2 = f32(f32(f32(-0.5) / s) / s)
    norm = f32(1.0 / (math.sqrt(2.0 * math.pi) * float(s)))
    taps = []
    x = f32(-radius)
    for _ in range(2 * radius + 1):
        x2 = f32(x * x)
        taps.append(f32(norm * f32(expf(float(f32(x2 * sigma2))))))
        x = f32(x + f32(1.0))
    total = f32(0.0)
    for v in taps:
        total = f32(total + v)
    fct = f32(f32(1.0) / total)
    return np.array([f32(v * fct) for v in taps], dtype=np.float32), radius


def gaussian_smooth(arr, sigma):
    """vigra.filters.gaussianSmoothing(arr, sigma) of a 3-D float32 array restated (TEST
    INFRASTRUCTURE ONLY, unpinned against vigra): separable, axes 0, 1, 2 in turn; per line
    out[x] = sum over i = x - r .. x + r (increasing) of tap[x - i] * src[reflect(i)], accumulated
    from 0 with separate float32 multiply and add, float32 between the axes; reflect mirrors
    without repeating the edge (BORDER_TREATMENT_REFLECT); every line must be longer than r
    (vigra's convolveLine precondition)."""
    taps, r = gaussian_taps(sigma)
    y = np.asarray(arr, dtype=np.float32)
    for ax in range(3):
        w = y.shape[ax]
        if w <= r:
            raise ValueError('convolveLine(): kernel longer than line')
        pad = [(r, r) if a == ax else (0, 0) for a in range(3)]
        p = np.pad(y, pad, mode='reflect')
        acc = np.zeros_like(y)
        for j in range(2 * r + 1):
            sl = [slice(None)] * 3
            sl[ax] = slice(j, j + w)
            acc = (acc + (taps[2 * r - j] * p[tuple(sl)]).astype(np.float32)).astype(np.float32)
        y = acc
    return y


def normalize_block(x):
    """vu.normalize (volume_utils.py:98-105), numpy as the reference runs it."""
    y = np.asarray(x).astype('float32')
    with np.errstate(invalid='ignore', divide='ignore'):
        y -= y.min()
        m = y.max()
        if m > 0:
            y /= m
    return y


def gaussian_smooth_blocks(inp, block_shape, sigma):
    """The sigma_prefilter front of block_components.py:160-163 per block (TEST INFRASTRUCTURE
    ONLY): normalize -> gaussian_smooth (restated vigra) -> (the second normalize is part of the
    labelling / threshold that follows)."""
    x = np.asarray(inp, dtype=np.float32)
    out = np.empty_like(x)
    grids = [range(0, s, b) for s, b in zip(x.shape, block_shape)]
    for z0 in grids[0]:
        for y0 in grids[1]:
            for x0 in grids[2]:
                bb = (slice(z0, z0 + block_shape[0]), slice(y0, y0 + block_shape[1]),
                      slice(x0, x0 + block_shape[2]))
                with np.errstate(invalid='ignore', over='ignore'):
                    out[bb] = gaussian_smooth(normalize_block(x[bb]), sigma)
    return out
