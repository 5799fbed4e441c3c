#!/usr/bin/env python3
"""Weighted minimax (Lawson) fits of erfc(x)/2 = e^{-x^2} P(x) on [0, X], x clamped at X: the
rcp-free alternative to the A&S 7.1.26 form of csrc/gelu_pk.h.  Prints the
max abs error of the fit and of its fp32 Horner evaluation over [0, 12] per degree.
    python tools/erfc_fit.py"""
import numpy as np
from scipy.special import erfc, erfcx
def fit(deg, X, iters=200):
    x = np.linspace(0, X, 4000)
    w = np.exp(-x*x)            # error weight: abs error of erfc(x)/2
    R = erfcx(x)/2
    V = np.vander(x, deg+1, increasing=True)
    lw = np.ones_like(x)
    best=None
    for it in range(iters):
        A = V * (w*lw)[:,None]; b = R*w*lw
        c = np.linalg.lstsq(A, b, rcond=None)[0]
        e = np.abs((V@c - R)*w)
        if best is None or e.max() < best[0]: best=(e.max(), c)
        lw = lw * (e/e.max() + 1e-3)**0.5   # Lawson-ish
        lw /= lw.max()
    return best
for X in (3.7, 3.9, 4.2):
  for deg in range(5, 11):
    err, c = fit(deg, X)
    # check with clamp over wide range in fp32 evaluation
    xx = np.linspace(0, 12, 200001)
    xc = np.minimum(xx, X).astype(np.float32)
    p = np.float32(c[-1])
    for k in range(deg-1, -1, -1): p = (p*xc + np.float32(c[k])).astype(np.float32)
    half = (np.exp(-xx*xx).astype(np.float32)*p)
    e2 = np.abs(half - erfc(xx)/2).max()
    print(f"X={X} deg={deg} fit={err:.2e} clampedfp32={e2:.2e}")
