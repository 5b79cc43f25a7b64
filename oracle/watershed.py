"""TEST INFRASTRUCTURE ONLY -- the checker of cc_watershed_from_seeds (never imported by the product).

Seeded watershed per block, restating what the reference's WatershedFromSeeds job does around
its (missing) watershed call (cluster_tools/watershed/watershed_from_seeds.py:143-273):
  * `_read_data`: the block's input normalized by vu.normalize (volume_utils.py:98-105); for 4-D
    input the channels channel_begin:channel_end normalized together, then np.mean / max / min
    over them (:127-139; read_data, pinned by goldens from the reference's own _read_data);
  * `_ws_block_masked`: blocks without a mask voxel are skipped, the input is set to 1 outside
    the mask and the result zeroed there;
  * `vu.watershed(input_, seeds=seeds.astype('uint32'), size_filter=0)`: volume_utils has no
    such function, so its behaviour is defined here (parity UNPINNED), 6-connected inside the
    block:
      cost(v)  = 0 for seeds, else min over paths from a seed of the max ordered f on the path,
                 the seed excluded: the least fixpoint of cost(v) = min_u max(cost(u), f(v));
      label(v) = the seed id for seeds, else the smallest label among the neighbours u with
                 max(cost(u), f(v)) == cost(v); 0 where no seed reaches v.
Both are computed here by Jacobi iteration to the fixpoint (numpy, small volumes only).
"""
import numpy as np

INF = np.uint64(0xFFFFFFFF)
NAN_ORD = np.uint64(0xFFFFFFFE)


def normalize(x):
    """vu.normalize (volume_utils.py:98-105), float32."""
    x = x.astype(np.float32)
    with np.errstate(invalid='ignore'):
        x = x - x.min()
        mx = x.max()
        if mx > 0:
            x = x / mx
    return x


def f2ord(f):
    u = f.astype(np.float32).view(np.uint32).astype(np.uint64)
    neg = (u >> np.uint64(31)) != 0
    o = np.where(neg, (~u) & np.uint64(0xFFFFFFFF), u | np.uint64(0x80000000))
    nan = (u & np.uint64(0x7FFFFFFF)) > np.uint64(0x7F800000)
    return np.where(nan, NAN_ORD, o).astype(np.uint64)


def _shifts(a, fill):
    """the six 6-neighbour views of `a` (padded with fill): a[v + d] for each d"""
    p = np.pad(a, 1, mode='constant', constant_values=fill)
    Z, Y, X = a.shape
    return [p[0:Z, 1:Y + 1, 1:X + 1], p[2:Z + 2, 1:Y + 1, 1:X + 1],
            p[1:Z + 1, 0:Y, 1:X + 1], p[1:Z + 1, 2:Y + 2, 1:X + 1],
            p[1:Z + 1, 1:Y + 1, 0:X], p[1:Z + 1, 1:Y + 1, 2:X + 2]]


def read_data_block(x4, channel_begin=0, channel_end=None, agg='mean'):
    """_read_data of a 4-D block (watershed_from_seeds.py:127-139): x4 = ds_in[:, bb] (C, ...);
    the channels channel_begin:channel_end normalized as ONE array (vu.normalize), then
    np.mean / np.max / np.min over axis 0 (float32)."""
    assert agg in ('mean', 'max', 'min')
    y = normalize(x4[channel_begin:channel_end])
    with np.errstate(invalid='ignore'):
        return getattr(np, agg)(y, axis=0)


def read_data(x4, block_shape, channel_begin=0, channel_end=None, agg='mean'):
    """read_data_block over the whole blocking -> (Z, Y, X) float32"""
    C, Z, Y, X = x4.shape
    out = np.zeros((Z, Y, X), dtype=np.float32)
    bz, by, bx = block_shape
    for z0 in range(0, Z, bz):
        for y0 in range(0, Y, by):
            for x0 in range(0, X, bx):
                bb = np.s_[z0:z0 + bz, y0:y0 + by, x0:x0 + bx]
                out[bb] = read_data_block(x4[(slice(None),) + bb], channel_begin, channel_end, agg)
    return out


def watershed_block(x, seeds, mask=None, normalized=False):
    """one block: float input, uint64 seeds (< 2^32 - 1), optional uint8 mask -> uint64 labels.
    normalized: x already holds _read_data's values (4-D input), not normalized again."""
    seeds = seeds.astype(np.uint64)
    assert int(seeds.max(initial=0)) < int(INF), 'seed ids must be < 2^32 - 1'
    if mask is not None and not mask.any():
        return np.zeros(x.shape, dtype=np.uint64)
    f = x.astype(np.float32).copy() if normalized else normalize(x)
    if mask is not None:
        f[mask == 0] = 1.0
    f = f2ord(f)
    is_seed = seeds != 0
    cost = np.where(is_seed, np.uint64(0), INF)
    while True:
        nb = np.minimum.reduce(_shifts(cost, INF))
        cand = np.where(nb == INF, INF, np.maximum(nb, f))
        new = np.where(is_seed, np.uint64(0), np.minimum(cost, cand))
        if np.array_equal(new, cost):
            break
        cost = new
    lab = np.where(is_seed, seeds, INF)
    cs = _shifts(cost, INF)
    preds = [(cu != INF) & (np.maximum(cu, f) == cost) & (cost != INF) & ~is_seed for cu in cs]
    while True:
        best = lab.copy()
        for ok, lu in zip(preds, _shifts(lab, INF)):
            best = np.where(ok, np.minimum(best, lu), best)
        if np.array_equal(best, lab):
            break
        lab = best
    out = np.where(lab == INF, np.uint64(0), lab).astype(np.uint64)
    if mask is not None:
        out[mask == 0] = 0
    return out


def watershed_from_seeds(x, seeds, block_shape, mask=None, channel_begin=0, channel_end=None, agg='mean'):
    """the job over the whole blocking (nifty blocking: blocks from the origin, clipped at the end);
    4-D x: channels first, each block read by _read_data (read_data_block)"""
    if x.ndim == 4:
        xn = read_data(x, block_shape, channel_begin, channel_end, agg)
        return _ws_blocks(xn, seeds, block_shape, mask, True)
    return _ws_blocks(x, seeds, block_shape, mask, False)


def _ws_blocks(x, seeds, block_shape, mask, normalized):
    out = np.zeros(x.shape, dtype=np.uint64)
    Z, Y, X = x.shape
    bz, by, bx = block_shape
    for z0 in range(0, Z, bz):
        for y0 in range(0, Y, by):
            for x0 in range(0, X, bx):
                bb = np.s_[z0:z0 + bz, y0:y0 + by, x0:x0 + bx]
                out[bb] = watershed_block(x[bb], seeds[bb], None if mask is None else mask[bb], normalized)
    return out
