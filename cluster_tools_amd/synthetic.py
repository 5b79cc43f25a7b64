"""Device-side synthetic inputs for bench.py.

ellipsoid_mask_device: the uint8 mask of config C4 -- 1 inside the centred ellipsoid with semi-axes
frac * extent -- for the z-slab [z0, z0 + nz) of a volume of shape gshape.  Same float64
formula and summation order as oracle/synth.py:ellipsoid_mask (the oracle is not imported here;
tests/test_boundary.py checks the two agree).  Built on the device in z-chunks (no host copy).
"""
import torch


def ellipsoid_mask_device(gshape, z0, nz, device, frac=0.45, chunk=64):
    Z, Y, X = (int(v) for v in gshape)
    f64 = dict(dtype=torch.float64, device=device)

    def axis_term(n, lo, cnt):
        c = (n - 1) / 2.0
        i = torch.arange(lo, lo + cnt, **f64)
        return ((i - c) / (frac * n)) ** 2

    ry = axis_term(Y, 0, Y).view(1, Y, 1)
    rx = axis_term(X, 0, X).view(1, 1, X)
    out = torch.empty((nz, Y, X), dtype=torch.uint8, device=device)
    for s in range(0, nz, chunk):
        e = min(nz, s + chunk)
        rz = axis_term(Z, z0 + s, e - s).view(-1, 1, 1)
        out[s:e] = ((rz + ry) + rx <= 1.0).to(torch.uint8)
    return out
