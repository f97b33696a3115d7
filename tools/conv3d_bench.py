#!/usr/bin/env python3
"""fsmi_conv3d_halo_x3 (split-precision halo conv, NCDHW) vs MIOpen (torch F.conv3d) on the 3D
cost-filtering layer shapes at cfg2 (D4=48, 120x160), per tile config.

    python tools/conv3d_bench.py [--reps 10] [--cfgs 5 6 7]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from foundationstereo_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--cfgs", type=int, nargs="*", default=[5, 6, 7])
ap.add_argument("--no-miopen", action="store_true")
a = ap.parse_args()
dev = torch.device("cuda:0")

# (name, cin, cout, (kd, k, k), D, H, W)
SHAPES = [
    ("stem.3x3x3", 28, 28, (3, 3, 3), 48, 120, 160),
    ("cls.3x3x3.28-14", 28, 14, (3, 3, 3), 48, 120, 160),
    ("cls.3x3x3.14-14", 14, 14, (3, 3, 3), 48, 120, 160),
    ("apc.1x3x3", 28, 28, (1, 3, 3), 48, 120, 160),
    ("apc.17x1x1", 28, 28, (17, 1, 1), 48, 120, 160),
    ("hg1.1x3x3", 56, 56, (1, 3, 3), 24, 60, 80),
    ("hg1.17x1x1", 56, 56, (17, 1, 1), 24, 60, 80),
    ("hg2.1x3x3", 112, 112, (1, 3, 3), 12, 30, 40),
    ("hg2.17x1x1", 112, 112, (17, 1, 1), 12, 30, 40),
    ("agg1.1x1x1", 112, 56, (1, 1, 1), 24, 60, 80),
]


def timeit(fn):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / a.reps


with torch.no_grad():
    for name, cin, cout, k, D, H, W in SHAPES:
        x = torch.randn(1, cin, D, H, W, device=dev)
        w = torch.randn(cout, cin, *k, device=dev) * 0.05
        b = torch.randn(cout, device=dev)
        pk = ops.PackedConv(w, mode="halo")
        fl = 2.0 * cin * cout * k[0] * k[1] * k[2] * D * H * W
        row = {"layer": name, "GFLOP": round(fl / 1e9, 1)}
        if not a.no_miopen:
            row["miopen_us"] = round(timeit(lambda: F.relu(F.conv3d(x, w, b, padding=tuple(q // 2 for q in k)))), 1)
        row["auto_us"] = round(timeit(lambda: ops.conv3d(x, pk, bias=b, act="relu")), 1)
        ref = F.relu(F.conv3d(x, w, b, padding=tuple(q // 2 for q in k)))
        for c in a.cfgs:
            row[f"cfg{c}_us"] = round(timeit(lambda: ops.conv3d(x, pk, bias=b, act="relu", cfg=c)), 1)
            y = ops.conv3d(x, pk, bias=b, act="relu", cfg=c)
            row[f"cfg{c}_err"] = float(((y - ref).abs().max() / ref.abs().max()).item())
        row["auto_TF"] = round(fl / row["auto_us"] / 1e6, 1)
        print(json.dumps(row), flush=True)
