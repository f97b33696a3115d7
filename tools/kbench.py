#!/usr/bin/env python3
"""Micro-benchmark of every libfsmi kernel at a workload's shapes (HIP events, many reps).

    python tools/kbench.py [--config cfg2] [--reps 50]

Prints per op: mean us, algorithmic MB moved and the resulting GB/s, so a
kernel change can be judged without a full bench run.  Inputs are random and
resident; outputs are allocated once per call by the op (as in the model).
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from foundationstereo_amd import ops  # noqa: E402

CFG = {"cfg2": (480, 640, 192, 128), "cfg2l": (480, 640, 192, 224), "cfg4": (384, 1248, 256, 224),
       "cfg5": (1024, 1536, 320, 224)}

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="cfg2")
ap.add_argument("--reps", type=int, default=50)
ap.add_argument("--levels", type=int, default=4)
a = ap.parse_args()
H, W, md, C = CFG[a.config]
H4, W4, D4 = H // 4, W // 4, md // 4
N = H4 * W4
L = a.levels
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)


def rnd(*s, scale=1.0):
    return torch.randn(*s, device=dev, generator=g) * scale


def timeit(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / a.reps


fl, fr = rnd(1, C, H4, W4), rnd(1, C, H4, W4)
A, Bm = rnd(1, 28, H4, W4), rnd(1, 28, H4, W4)
Wg = rnd(28, 8, scale=0.3)
wt = rnd(28, C, scale=0.1)
bias = rnd(28)
vol = rnd(1, 28, D4, H4, W4)
vpyr = ops.volume_pyramid(vol, L)
cpyr = ops.allpairs_corr(fl, fr, L)
# piecewise-smooth disparity (a slanted plane + small noise), like a real scene; fully random
# per-pixel disparities make every lookup load a divergent gather (reported separately)
ramp = torch.linspace(0.2 * D4, 0.8 * D4, W4, device=dev).view(1, 1, 1, W4).expand(1, 1, H4, W4)
disp = (ramp + 0.3 * torch.rand(1, 1, H4, W4, device=dev, generator=g)).contiguous()
disp_rand = torch.rand(1, 1, H4, W4, device=dev, generator=g) * D4
logits = rnd(1, D4, H4, W4)
mask_logits = rnd(1, 9, H, W)
Hd, Cx = 128, 384
zr = rnd(1, 2 * Hd, H4, W4)
h = rnd(1, Hd, H4, W4)
x = rnd(1, Cx, H4, W4)
q = rnd(1, Hd, H4, W4)
att = torch.rand(1, 1, H4, W4, device=dev, generator=g)
K = 9
res = {}
cases = {
    "gwc_volume": (lambda: ops.gwc_volume(fl, fr, D4, 8), 4 * (2 * C * N + 8 * D4 * N)),
    "comb_two_pass": (lambda: ops.comb_volume_stem(fl, fr, A, Bm, Wg, D4, True), 4 * N * (2 * C + 56 + 28 * D4)),
    "comb_one_pass": (lambda: ops.comb_volume_stem(fl, fr, A, Bm, Wg, D4, False), 4 * N * (2 * C + 56 + 28 * D4)),
    "pointwise_proj": (lambda: ops.pointwise_proj(fl, wt, bias), 4 * N * (C + 28)),
    "allpairs_corr": (lambda: ops.allpairs_corr(fl, fr, L), 4 * (2 * C * N + sum(N * (W4 >> i) for i in range(L)))),
    "allpairs_corr_1pass": (lambda: ops.allpairs_corr(fl, fr, L, False),
                            4 * (2 * C * N + sum(N * (W4 >> i) for i in range(L)))),
    "geo_lookup_randdisp": (lambda: ops.geo_lookup(vpyr, cpyr, disp_rand, 4),
                            4 * N * (1 + L * 29 * (K + 1) + L * K * 29)),
    "volume_pyramid": (lambda: ops.volume_pyramid(vol, L),
                       4 * (28 * D4 * N + sum(28 * (D4 >> i) * N for i in range(1, L)))),
    "geo_lookup": (lambda: ops.geo_lookup(vpyr, cpyr, disp, 4),
                   4 * N * (1 + L * 29 * (K + 1) + L * K * 29)),
    "softmax_regression": (lambda: ops.softmax_regression(logits), 4 * N * (D4 + 1)),
    "softmax_upsample": (lambda: ops.softmax_context_upsample(disp, mask_logits, 4.0), 4 * (N + 10 * 16 * N)),
    "gru_reset": (lambda: ops.gru_reset(zr, zr, h, x), 4 * N * (2 * Hd + Hd + Cx + 2 * (Hd + Cx))),
    "gru_blend": (lambda: ops.gru_blend(zr, zr, q, q, h, att), 4 * N * (2 * Hd + 2 * Hd + Hd + 1 + Hd)),
}
for name, (fn, nbytes) in cases.items():
    us = timeit(fn)
    res[name] = {"us": round(us, 2), "MB": round(nbytes / 1e6, 2), "GBps": round(nbytes / us / 1e3, 1)}
    print(f"{name:20s} {us:9.2f} us {nbytes / 1e6:9.2f} MB {nbytes / us / 1e3:8.1f} GB/s", flush=True)
print(json.dumps({"config": a.config, "levels": L, "kernels": res}))
