"""Synthetic boundary-map generator, numpy restatement (TEST INFRASTRUCTURE).

This file is part of the oracle: only tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py may use it.  The product generates the same volume
on the GPU (`cc_generate_boundary_map`, cluster_tools_amd/csrc/cc_generate.hip);
tests check the two are bit-identical.

Definition (integer-only so CPU and GPU agree bit for bit):
  * jittered Voronoi seeds, one per pitch-32 cell; cell (cz,cy,cx) (each >= -1)
    has key ((cz+1)<<42)|((cy+1)<<21)|(cx+1), h = splitmix64(seed ^ key) and seed
    point (32cz + h&31, 32cy + (h>>5)&31, 32cx + (h>>10)&31);
  * d1 <= d2: the two smallest squared distances from the voxel to the seeds of
    the 3x3x3 cells around its own cell;
  * membrane m = max(0, 255 - (d2 - d1));
  * noise n = splitmix64((seed + NOISE_SALT) ^ vkey) % 33 - 16 with
    vkey = (z<<42)|(y<<21)|x (independent of the volume shape, so any sub-box of
    a volume equals the same sub-box generated on its own);
  * q = clamp(m + n, 0, 255); value = float32(q) / 256 (exact);
  * continuous variant (dither=True): d = (nh >> 16) & 0xFFFF and value = float32(q * 2^16 + d)
    / 2^24 (exact), i.e. q / 256 plus a deterministic sub-2^-8 dither, so block extremes and
    threshold crossings are no longer quantized.
"""
import numpy as np

PITCH = 32
MASTER_SEED = 0x5EED
NOISE_SALT = 0x5851F42D4C957F2D
_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x):
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over='ignore'):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def boundary_q(shape, origin=(0, 0, 0), seed=MASTER_SEED, with_dither=False):
    """uint8 membrane strength q for the box [origin, origin+shape) (and the uint16 dither)."""
    Z, Y, X = shape
    z = np.arange(origin[0], origin[0] + Z, dtype=np.int64)[:, None, None]
    y = np.arange(origin[1], origin[1] + Y, dtype=np.int64)[None, :, None]
    x = np.arange(origin[2], origin[2] + X, dtype=np.int64)[None, None, :]
    cz, cy, cx = z // PITCH, y // PITCH, x // PITCH
    big = np.int64(1) << 62
    d1 = np.full(shape, big, dtype=np.int64)
    d2 = np.full(shape, big, dtype=np.int64)
    seed64 = np.uint64(seed)
    for dz in (-1, 0, 1):
        for dy in (-1, 0, 1):
            for dx in (-1, 0, 1):
                nz, ny, nx = cz + dz, cy + dy, cx + dx
                key = (((nz + 1).astype(np.uint64) << np.uint64(42))
                       | ((ny + 1).astype(np.uint64) << np.uint64(21))
                       | (nx + 1).astype(np.uint64))
                h = splitmix64(seed64 ^ key)
                sz = nz * PITCH + (h & np.uint64(31)).astype(np.int64)
                sy = ny * PITCH + ((h >> np.uint64(5)) & np.uint64(31)).astype(np.int64)
                sx = nx * PITCH + ((h >> np.uint64(10)) & np.uint64(31)).astype(np.int64)
                d = (z - sz) ** 2 + (y - sy) ** 2 + (x - sx) ** 2
                d2 = np.where(d < d1, d1, np.minimum(d2, d))
                d1 = np.minimum(d1, d)
    m = np.maximum(0, 255 - (d2 - d1))
    vkey = ((z.astype(np.uint64) << np.uint64(42)) | (y.astype(np.uint64) << np.uint64(21))
            | x.astype(np.uint64))
    with np.errstate(over='ignore'):
        nh = splitmix64((seed64 + np.uint64(NOISE_SALT)) ^ vkey)
    n = (nh % np.uint64(33)).astype(np.int64) - 16
    q = np.clip(m + n, 0, 255).astype(np.uint8)
    if with_dither:
        return q, ((nh >> np.uint64(16)) & np.uint64(0xFFFF)).astype(np.uint32)
    return q


def boundary_map(shape, origin=(0, 0, 0), seed=MASTER_SEED, dither=False):
    """float32 boundary map in [0, 255/256] (dither: the continuous variant, below 1)."""
    if dither:
        q, d = boundary_q(shape, origin, seed, with_dither=True)
        return (q.astype(np.uint32) * np.uint32(65536) + d).astype(np.float32) / np.float32(1 << 24)
    return boundary_q(shape, origin, seed).astype(np.float32) / np.float32(256)


def ellipsoid_mask(shape, frac=0.45):
    """uint8 mask: 1 inside the centred ellipsoid with semi-axes frac*extent.

    Integer test: sum_a ((2*p_a + 1 - n_a) * S/n_a)^2 <= (2*frac*S)^2 style is
    avoided; we use float64, which is exact enough for the small shapes it is
    used on and identical on every host (the GPU never generates masks)."""
    idx = np.indices(shape, dtype=np.float64)
    r = 0.0
    for a, n in enumerate(shape):
        c = (n - 1) / 2.0
        r = r + ((idx[a] - c) / (frac * n)) ** 2
    return (r <= 1.0).astype(np.uint8)
