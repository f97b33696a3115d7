#!/usr/bin/env python3
"""Hourglass Conv3d(k3, s2, p1) + BN + LeakyReLU at cfg2's shapes: MIOpen/CK (torch) vs the stride-2
halo tiles per cfg / split, graph-timed.  GPU box: python tools/s2_bench.py"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from foundationstereo_amd import ops  # noqa: E402

dev = torch.device("cuda:0")


def gtime(f, reps=10):
    f()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            f()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) * 1e3 / reps, 1)


with torch.no_grad():
    for cin, cout, D, H, W in ((28, 56, 48, 120, 160), (56, 112, 24, 60, 80), (112, 168, 12, 30, 40)):
        x = torch.randn(1, cin, D, H, W, device=dev)
        w = torch.randn(cout, cin, 3, 3, 3, device=dev) * 0.05
        sc, sh = torch.rand(cout, device=dev) + 0.5, torch.randn(cout, device=dev)
        pk = ops.PackedConv(w * sc.view(-1, 1, 1, 1, 1), mode="halo")
        row = {"shape": f"{cin}->{cout} @{D}x{H}x{W}",
               "torch_us": gtime(lambda: F.leaky_relu(F.conv3d(x, w, stride=2, padding=1)
                                                      * sc.view(1, -1, 1, 1, 1) + sh.view(1, -1, 1, 1, 1), 0.01))}
        for c in (-1, 4, 5, 7, 10):
            for ns in ((1, 2, 3, 4) if c >= 0 else (-1,)):
                row[f"cfg{c}_s{ns}_us"] = gtime(lambda: ops.conv3d(x, pk, bias=sh, act="leaky", stride=2, cfg=c,
                                                                     nsplit=ns))
        print(json.dumps(row), flush=True)
