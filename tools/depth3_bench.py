#!/usr/bin/env python3
"""The (3, 3, 3) volume convs of the 3D filter at cfg2 (and cfg5's full-resolution stem) on the
depth-blocked tile (cfg 31) vs the tuning table's choice, each the mean over a replayed graph of
10 launches, with the max |diff| between the two.  GPU box: python tools/depth3_bench.py [--only NAME]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from foundationstereo_amd import ops  # noqa: E402

dev = torch.device("cuda:0")


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) * 1e3 / reps, 1)


SHAPES = [(28, 28, 48, 120, 160, "leaky", "stem 3^3"), (28, 14, 48, 120, 160, "leaky", "classifier 28->14"),
          (14, 14, 48, 120, 160, "leaky", "classifier 14->14"), (56, 56, 24, 60, 80, "leaky", "hourglass 56"),
          (28, 28, 80, 256, 384, "leaky", "cfg5 full-res stem")]
ONLY = sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else None   # layer-name prefix
with torch.no_grad():
    for cin, cout, D, H, W, act, name in SHAPES:
        if ONLY and not name.startswith(ONLY):
            continue
        x = torch.randn(1, cin, D, H, W, device=dev)
        pk = ops.PackedConv(torch.randn(cout, cin, 3, 3, 3, device=dev) * 0.05, mode="halo")
        b = torch.randn(cout, device=dev)
        o1 = torch.empty(1, cout, D, H, W, device=dev)
        ta = timed(lambda: o1.copy_(ops.conv3d(x, pk, bias=b, act=act)))
        t31 = timed(lambda: o1.copy_(ops.conv3d(x, pk, bias=b, act=act, cfg=31)))
        a1, a2 = ops.conv3d(x, pk, bias=b, act=act), ops.conv3d(x, pk, bias=b, act=act, cfg=31)
        flops = 2 * cin * cout * 27 * D * H * W
        print(json.dumps({"layer": name, "table_us": ta, "cfg31_us": t31, "cfg31_TFLOPs": round(flops / t31 / 1e6, 1),
                          "table_TFLOPs": round(flops / ta / 1e6, 1),
                          "max_abs_diff": float((a1 - a2).abs().max())}), flush=True)
