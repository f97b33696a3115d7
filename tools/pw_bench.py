#!/usr/bin/env python3
"""Times the pointwise LDS-DMA tiles (cfg 24-26, conv_pw.hip) against the table entry on the cfg2
loop's 1x1 shapes: every (cfg, split) -> us.  GPU box: python tools/pw_bench.py [--reps 20]"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from foundationstereo_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--cfgs", type=int, nargs="*", default=[24, 25, 26, 27, 28, 29])
a = ap.parse_args()
dev = torch.device("cuda:0")
SHAPES = [(512, 128, 120, 160), (1044, 256, 120, 160), (128, 512, 120, 160), (512, 256, 120, 160),
          (512, 128, 60, 80), (512, 256, 60, 80), (384, 128, 30, 40)]


def timeit(fn):                                    # reps calls in one replayed hipGraph
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(a.reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) * 1e3 / a.reps, 1)


with torch.no_grad():
    for cin, cout, H, W in SHAPES:
        x = torch.randn(1, cin, H, W, device=dev)
        pk = ops.PackedConv(torch.randn(cout, cin, 1, 1, device=dev) * 0.05, mode="halo")
        b = torch.randn(cout, device=dev)
        row = {"shape": f"{cin}->{cout} @{H}x{W}", "table": timeit(lambda: ops.conv2d([x], pk, bias=b, act="relu"))}
        for c in a.cfgs:
            for s in (1, 2, 3, 4):
                if s <= (cin + 31) // 32 // 2 or s == 1:
                    row[f"{c}/{s}"] = timeit(lambda: ops.conv2d([x], pk, bias=b, act="relu", cfg=c, nsplit=s))
        best = min((v, k) for k, v in row.items() if k not in ("shape",))
        row["best"] = best
        print(json.dumps(row), flush=True)
