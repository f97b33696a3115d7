#!/usr/bin/env python3
"""Hourglass ConvTranspose3d(k4, s2, p1) + BN + LeakyReLU at cfg2's shapes: MIOpen/CK (torch) vs the
2x2x2 phase tiles per cfg, graph-timed.  GPU box: python tools/up3d_bench.py"""
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
    for cin, cout, D, H, W in ((168, 112, 6, 15, 20), (112, 56, 12, 30, 40), (56, 28, 24, 60, 80)):
        x = torch.randn(1, cin, D, H, W, device=dev)
        w = torch.randn(cin, cout, 4, 4, 4, device=dev) * 0.05
        sc, sh = torch.rand(cout, device=dev) + 0.5, torch.randn(cout, device=dev)
        packs = ops.pack_deconv_phases(w, sc)
        row = {"shape": f"{cin}->{cout} @{D}x{H}x{W}",
               "torch_us": gtime(lambda: F.leaky_relu(F.conv_transpose3d(x, w, stride=2, padding=1)
                                                      * sc.view(1, -1, 1, 1, 1) + sh.view(1, -1, 1, 1, 1), 0.01))}
        for c in (2, 3, 5, 6, 7):
            row[f"cfg{c}_us"] = gtime(lambda: ops.conv3d_up2(x, packs, bias=sh, act="leaky", cfg=c))
        print(json.dumps(row), flush=True)
