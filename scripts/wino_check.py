"""Derives the Winograd F(m, r) transform matrices by Toom-Cook (exact
rationals) and measures the fp32 error of F(2x2, 5x5) against an fp64
reference on random data, next to a direct fp32 sum (docs/ACCURACY.md,
csrc/kernels/wino.h).    python scripts/wino_check.py"""
from fractions import Fraction as Fr
import numpy as np, itertools

def toom_cook(m, r, pts):
    # pts: alpha-1 finite points + infinity; returns AT (m x a), G (a x r), BT (a x a) (Lavin & Gray)
    a = m + r - 1
    assert len(pts) == a - 1
    f = [Fr(p) for p in pts]
    # Vandermonde-based construction (as in wincnn)
    # A^T: m x a ; rows i: p_j^i for finite, last col [0..0,1]
    AT = [[f[j]**i for j in range(a-1)] + [Fr(1) if i == m-1 else Fr(0)] for i in range(m)]
    # G: a x r ; rows j: p_j^k / N_j  where N_j = prod_{l!=j}(p_j-p_l); last row [0..0,1]
    N = []
    for j in range(a-1):
        n = Fr(1)
        for l in range(a-1):
            if l != j: n *= (f[j]-f[l])
        N.append(n)
    G = [[f[j]**k / N[j] for k in range(r)] for j in range(a-1)] + [[Fr(1) if k == r-1 else Fr(0) for k in range(r)]]
    # B^T: a x a : from polynomial M(x) = prod (x - p_j); row j: coefficients of M(x)/(x-p_j) ; last row coeffs of M(x)
    def polymul(p, q):
        out = [Fr(0)]*(len(p)+len(q)-1)
        for i,x in enumerate(p):
            for j,y in enumerate(q): out[i+j] += x*y
        return out
    BT = []
    for j in range(a-1):
        poly = [Fr(1)]
        for l in range(a-1):
            if l != j: poly = polymul(poly, [-f[l], Fr(1)])
        BT.append(poly + [Fr(0)]*(a - len(poly)))
    poly = [Fr(1)]
    for l in range(a-1): poly = polymul(poly, [-f[l], Fr(1)])
    BT.append(poly)
    return AT, G, BT

def to_np(M, dt=np.float64): return np.array([[float(x) for x in row] for row in M], dt)

def check(m, r, pts, dt=np.float32, trials=200):
    AT, G, BT = toom_cook(m, r, pts)
    AT_, G_, BT_ = to_np(AT), to_np(G), to_np(BT)
    a = m + r - 1
    rs = np.random.RandomState(0)
    # 1D check exact in f64
    d = rs.randn(a); g = rs.randn(r)
    direct = np.array([sum(d[i+k]*g[k] for k in range(r)) for i in range(m)])
    wino = AT_ @ ((G_ @ g) * (BT_ @ d))
    assert np.allclose(direct, wino), (direct, wino)
    # 2D fp32 error vs f64 with channel sum C=32
    C = 32; errs = []
    ATf, Gf, BTf = to_np(AT, dt), to_np(G, dt), to_np(BT, dt)
    for t in range(trials):
        d = rs.randn(C, a, a); g = rs.randn(C, r, r) * 0.1
        ref = np.zeros((m, m))
        for c in range(C):
            for i in range(m):
                for j in range(m):
                    ref[i, j] += (d[c, i:i+r, j:j+r] * g[c]).sum()
        dd = d.astype(dt); gg = g.astype(dt)
        U = np.einsum('ik,ckl,jl->cij', Gf, gg, Gf).astype(dt)
        V = np.einsum('ik,ckl,jl->cij', BTf, dd, BTf).astype(dt)
        Mm = (U * V).sum(0, dtype=dt)
        Y = (ATf @ Mm @ ATf.T).astype(dt)
        # direct fp32
        dref = np.zeros((m, m), dt)
        for c in range(C):
            for i in range(m):
                for j in range(m):
                    dref[i, j] += (dd[c, i:i+r, j:j+r] * gg[c]).sum(dtype=dt)
        scale = np.abs(ref).max() + 1e-30
        errs.append((np.abs(Y - ref).max() / scale, np.abs(dref - ref).max() / scale))
    e = np.array(errs)
    return e[:, 0].mean(), e[:, 0].max(), e[:, 1].mean(), e[:, 1].max()

for pts in ([0, 1, -1, 2, -2], [0, 1, -1, Fr(1,2), -Fr(1,2)], [0, 1, -1, 2, Fr(-1,2)]):
    print(pts, "wino mean/max, direct mean/max:", check(2, 5, pts))
AT, G, BT = toom_cook(2, 5, [0, 1, -1, Fr(1,2), -Fr(1,2)])
for n, M in (("AT", AT), ("G", G), ("BT", BT)):
    print(n); [print("  ", [str(x) for x in row]) for row in M]
print("=== chosen points [0,1,-1,2,-1/2]")
AT, G, BT = toom_cook(2, 5, [0, 1, -1, 2, Fr(-1,2)])
for n, M in (("AT", AT), ("G", G), ("BT", BT)):
    print(n); [print("  ", [str(x) for x in row]) for row in M]
# 1D wgrad form F(5,2): output 5 from input 6 and filter 2
AT5, G5, BT5 = toom_cook(5, 2, [0, 1, -1, 2, Fr(-1,2)])
for n, M in (("AT5", AT5), ("G5", G5), ("BT5", BT5)):
    print(n); [print("  ", [str(x) for x in row]) for row in M]
