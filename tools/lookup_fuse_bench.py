#!/usr/bin/env python3
"""geo_lookup + convc1 (1x1, 1044 -> 256, ReLU) vs the fused fsmi_conv1x1_lookup at cfg2's shape,
graph-timed.  GPU box: python tools/lookup_fuse_bench.py"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from foundationstereo_amd import ops  # noqa: E402

dev = torch.device("cuda:0")


def gtime(f, reps=20):
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
    for B in (1, 4):
        L, Cv, D, H, W = 4, 28, 48, 120, 160
        vol = torch.randn(B, Cv, D, H, W, device=dev)
        fl, fr = torch.randn(B, 128, H, W, device=dev), torch.randn(B, 128, H, W, device=dev)
        corr = ops.allpairs_corr(fl, fr, L)
        pyr = ops.volume_pyramid(vol, L)
        disp = torch.rand(B, 1, H, W, device=dev) * D
        w = torch.randn(256, L * 9 * (Cv + 1), 1, 1, device=dev) * 0.05
        b = torch.randn(256, device=dev)
        pk, pkf = ops.PackedConv(w, mode="halo"), ops.pack_lookup_conv(w, L, Cv, 4)
        lk = ops.geo_lookup(pyr, corr, disp, 4)
        row = {"B": B, "lookup_us": gtime(lambda: ops.geo_lookup(pyr, corr, disp, 4, out=lk)),
               "convc1_us": gtime(lambda: ops.conv2d([lk], pk, bias=b, act="relu"))}
        for s in (1, 2, 3, 4, 6):
            row[f"fused_s{s}_us"] = gtime(lambda: ops.conv1x1_lookup(pyr, corr, disp, 4, pkf, bias=b, act="relu",
                                                                    nsplit=s))
        print(json.dumps(row), flush=True)
