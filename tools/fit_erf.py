#!/usr/bin/env python3
"""Coefficients of the branch-free erf used by the GELU epilogues (csrc/conv_halo.h gelu_fast):

    |z| <  1:  erf(z) = z * P(z^2)                         P: degree NP in t = z^2
    |z| >= 1:  erf(|z|) = 1 - exp(-z^2) * R(|z|)          R ~ erfcx on [1, 4]; 1 beyond 3.92

Least squares on Chebyshev nodes (relative error weights) in float64, then the max error of the
float32 evaluation (Horner with fmaf, numpy float32 emulation) against math.erf over a dense grid,
in units in the last place of the float32 result.  Prints C++ initialisers.  CPU only:

    python tools/fit_erf.py [--np 6] [--nr 10]
"""
import argparse
import math

import numpy as np

ap = argparse.ArgumentParser()
ap.add_argument("--np", type=int, default=6)
ap.add_argument("--nr", type=int, default=10)
a = ap.parse_args()


def cheb_nodes(lo, hi, n):
    k = np.arange(n)
    return 0.5 * (lo + hi) + 0.5 * (hi - lo) * np.cos(np.pi * (k + 0.5) / n)


def fit(x, y, deg, w):
    V = np.vander(x, deg + 1, increasing=True)
    c, *_ = np.linalg.lstsq(V * w[:, None], y * w, rcond=None)
    return c


erf = np.vectorize(math.erf)
erfc = np.vectorize(math.erfc)

# P(t) = erf(sqrt t) / sqrt t on t in [0, 1]
t = cheb_nodes(0.0, 1.0, 4000)
yp = erf(np.sqrt(t)) / np.sqrt(t)
cp = fit(t, yp, a.np, 1.0 / yp)
# R(z) = erfc(z) exp(z^2) on z in [1, 4]
z = cheb_nodes(1.0, 4.0, 4000)
yr = erfc(z) * np.exp(z * z)
cr = fit(z, yr, a.nr, 1.0 / yr)

f32 = np.float32


def horner32(c, x):
    r = np.full_like(x, f32(c[-1]))
    for ci in c[-2::-1]:
        r = (r.astype(np.float64) * x + f32(ci)).astype(f32)   # fmaf: one rounding
    return r


def erf32(zz):
    zz = zz.astype(f32)
    az = np.abs(zz)
    tt = (zz * zz).astype(f32)
    small = (zz.astype(np.float64) * horner32(cp, tt)).astype(f32)
    azc = np.minimum(az, f32(4.0))
    e = np.exp(-(tt.astype(np.float64))).astype(f32)              # device: v_exp_f32 of -t*log2(e)
    big = (1.0 - e.astype(np.float64) * horner32(cr, azc)).astype(f32)
    big = np.copysign(big, zz)
    return np.where(az < 1.0, small, big)


zs = np.concatenate([np.linspace(-6, 6, 2_000_001), np.geomspace(1e-30, 1, 20001)]).astype(f32)
got = erf32(zs).astype(np.float64)
ref = erf(zs.astype(np.float64))
ulp = np.spacing(np.abs(ref).astype(f32)).astype(np.float64)
err = np.abs(got - ref) / ulp
print(f"max error {err.max():.3f} ulp at z = {zs[err.argmax()]:.6g}; mean {err.mean():.3f}")
print("P:", ", ".join(f"{float(f32(c)):.9e}f" for c in cp))
print("R:", ", ".join(f"{float(f32(c)):.9e}f" for c in cr))
