#!/usr/bin/env python3
"""SelectiveConvGRU's small (1x1) branch at the cfg2 loop's three levels: the fused kernel
(ops.gru_small, csrc/gru_small.hip) vs the two gate convs it replaces (zr with the z / r*h epilogue,
then convq with the blend epilogue, at their tuned tiles), each the mean over a replayed graph of
20 launches, plus the fused result's max |diff| from the two-conv path.
GPU box: python tools/gru_small_bench.py"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from foundationstereo_amd import ops, synth  # noqa: E402
from foundationstereo_amd.update import RaftConvGRU, _packed  # noqa: E402

dev = torch.device("cuda:0")


def timed(fn, reps=20):
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
    for _ in range(3):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) * 1e3 / (3 * reps), 2)


with torch.no_grad():
    for K, H, W in ((512, 120, 160), (512, 60, 80), (384, 30, 40)):
        Hd = 128
        gru = RaftConvGRU(Hd, K - Hd, 1)
        synth.init_module_(gru, seed=7)
        gru = gru.to(dev).eval()
        hx = torch.randn(1, K, H, W, device=dev).abs()
        xc = torch.randn(1, K - Hd, H, W, device=dev).abs()
        h = torch.randn(1, Hd, H, W, device=dev)
        att = torch.rand(1, 1, H, W, device=dev)
        pkzr, bzr = _packed(gru.convz, gru.convr)
        pkq, bq = _packed(gru.convq)
        o1, o2 = torch.empty_like(h), torch.empty_like(h)
        z, rh = torch.empty_like(h), torch.empty_like(h)

        def two():
            ops.conv2d_gate([hx], pkzr, bzr, "zr", h=h, z=z, rh=rh)
            ops.conv2d_gate([rh, xc], pkq, bq, "blend_small", h=h, z=z, att=att, out=o2)

        fused = timed(lambda: ops.gru_small(hx, xc, h, att, pkzr, bzr, pkq, bq, out=o1))
        t2 = timed(two)
        flops = 2 * K * 3 * Hd * H * W
        print(json.dumps({"shape": f"K{K} {H}x{W}", "fused_us": fused, "two_conv_us": t2,
                          "fused_TFLOPs": round(flops / fused / 1e6, 1), "two_TFLOPs": round(flops / t2 / 1e6, 1),
                          "max_abs_diff": float((o1 - o2).abs().max())}), flush=True)
