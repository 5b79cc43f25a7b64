# tools/seams_sim.py -- CPU count of k_seams' work per tile: contact run starts walked, after the per-lane (la, lb)
# filter (= hash probes), distinct keys per tile (= emits).  Intra-block face seams only.
import sys, numpy as np, scipy.ndimage as ndi
sys.path.insert(0, '/root/repo')
from oracle import oracle as O
TZ, TY, TX = 16, 32, 64
Z, Y, X = 64, 512, 512
x = O.boundary_map((Z, Y, X), origin=(256, 512, 1024))
fg = x > 0.5
print('fg frac', fg.mean())
st = np.ones((3, 3, 3), bool)
lab = np.zeros(fg.shape, np.int32)
for z in range(0, Z, TZ):
    for y in range(0, Y, TY):
        for xx in range(0, X, TX):
            l, n = ndi.label(fg[z:z+TZ, y:y+TY, xx:xx+TX], structure=st)
            lab[z:z+TZ, y:y+TY, xx:xx+TX] = l
def sh(v, dx):  # bit x := bit x + dx, rows as bool arrays along axis -1
    out = np.zeros_like(v)
    if dx > 0: out[..., :-1] = v[..., 1:]
    elif dx < 0: out[..., 1:] = v[..., :-1]
    else: out = v.copy()
    return out
def seam(Aab, Bab, Ka, Kb):
    # Aab: own rows (R, W) bool; Bab neighbour rows; Ka/Kb ids per voxel
    R, W = Aab.shape
    walked = probes = 0
    keys = set()
    for r in range(R):
        A = Aab[r]; B0 = Bab[r]
        Am = Aab[r-1] if r > 0 else np.zeros(W, bool); Ap = Aab[r+1] if r+1 < R else np.zeros(W, bool)
        Bm = Bab[r-1] if r > 0 else np.zeros(W, bool); Bp = Bab[r+1] if r+1 < R else np.zeros(W, bool)
        if not A.any(): continue
        la = lb = None
        for dr in (-1, 0, 1):
            B = Bm if dr < 0 else Bp if dr > 0 else B0
            Ad = Am if dr < 0 else Ap
            rb = r + dr
            for dx in (-1, 0, 1):
                C = A & sh(B, dx)
                if dx: C &= ~(sh(A, dx) | B)
                if dr: C &= ~(Ad | sh(B0, dx))
                m0 = C & ~np.concatenate([[False], C[:-1]])
                if not dr and not dx: m0 &= ~(Am & Bm)
                for xi in np.nonzero(m0)[0]:
                    walked += 1
                    ka = Ka[r, xi]; kb = Kb[rb, xi + dx]
                    if ka == la and kb == lb: continue
                    la, lb = ka, kb
                    probes += 1
                    keys.add(((dr, dx), ka, kb) if False else (ka, kb))
    return walked, probes, len(keys)
tot = np.zeros(3, int); per = []
for z in range(TZ, Z, TZ):
    for y in range(0, Y, TY):
        for xx in range(0, X, TX):
            # z seam: own plane z (rows y, bits x) vs neighbour plane z-1
            w = seam(fg[z, y:y+TY, xx:xx+TX], fg[z-1, y:y+TY, xx:xx+TX], lab[z, y:y+TY, xx:xx+TX], lab[z-1, y:y+TY, xx:xx+TX])
            per.append(w); tot += w
print('z seams: tiles', len(per), 'walked/probes/distinct per tile', tot / len(per))
per = []; tot[:] = 0
for z in range(0, Z, TZ):
    for y in range(TY, Y, TY):
        for xx in range(0, X, TX):
            w = seam(fg[z:z+TZ, y, xx:xx+TX], fg[z:z+TZ, y-1, xx:xx+TX], lab[z:z+TZ, y, xx:xx+TX], lab[z:z+TZ, y-1, xx:xx+TX])
            per.append(w); tot += w
print('y seams: per tile', tot / len(per))
per = []; tot[:] = 0
for z in range(0, Z, TZ):
    for y in range(0, Y, TY):
        for xx in range(TX, X, TX):
            w = seam(fg[z:z+TZ, y:y+TY, xx], fg[z:z+TZ, y:y+TY, xx-1], lab[z:z+TZ, y:y+TY, xx], lab[z:z+TZ, y:y+TY, xx-1])
            per.append(w); tot += w
print('x seams: per tile', tot / len(per))
