#!/usr/bin/env python3
"""geo_lookup at cfg2 (B=1, MALL-resident pyramid) and cfg3's per-GPU batch (B=4, off-MALL): mean
launch time over a replayed graph of 20 launches and algorithmic GB/s (SURVEY §8d bytes).
Library variant from FSMI_LIB.  GPU box: python tools/lookup_bench.py"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from foundationstereo_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
L, Cv, r = 4, 28, 4
res = {"lib": os.path.basename(os.environ.get("FSMI_LIB", "libfsmi.so"))}
with torch.no_grad():
    for B, H, W, D in ((1, 120, 160, 48), (4, 120, 160, 48)):
        gen = torch.Generator().manual_seed(1)
        vol = torch.randn(B, Cv, D, H, W, generator=gen).to(dev)
        fl, fr = (torch.randn(B, 128, H, W, generator=gen).to(dev) for _ in range(2))
        corr = ops.allpairs_corr(fl, fr, L)
        pyr = ops.volume_pyramid(vol, L)
        # a smooth disparity field, as the loop sees (neighbouring pixels read neighbouring taps)
        hh = torch.arange(H).view(1, 1, H, 1).float()
        ww = torch.arange(W).view(1, 1, 1, W).float()
        disp = (0.2 * D + 0.5 * D * ww / W + 2.0 * torch.sin(hh / 7.0) + 0.37 * torch.rand(B, 1, 1, 1, generator=gen)
                ).expand(B, 1, H, W).contiguous().to(dev)
        ops.geo_lookup(pyr, corr, disp, r)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        reps = 20
        with torch.cuda.graph(g):
            for _ in range(reps):
                ops.geo_lookup(pyr, corr, disp, r)
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / (3 * reps)
        N = H * W
        byts = 4 * B * N * (1 + L * (Cv + 1) * (2 * r + 2) + L * (Cv + 1) * (2 * r + 1))
        res[f"B{B}_us"] = round(us, 2)
        res[f"B{B}_TBs"] = round(byts / us / 1e6, 3)
print(json.dumps(res), flush=True)
