#!/usr/bin/env python3
"""DispHead's EdgeNeXt MLP at cfg2's shape (1, 128, 120, 160): the fused kernel (ops.edgenext_mlp)
vs the two 1x1 convs it replaces (pwconv1 + GELU, pwconv2 + gamma + residual), each timed as the
mean over a replayed graph of 20 launches; then one eager fused launch with the debug phase stamps
(fsmi_debug_conv_timestamps): mean per-block phase durations in us and the launch span.
GPU box: python tools/mlp_bench.py"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from foundationstereo_amd import _lib, ops, synth, update  # noqa: E402
from foundationstereo_amd.submodule import EdgeNextConvEncoder  # noqa: E402

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
    return e0.elapsed_time(e1) * 1e3 / (3 * reps)


res = {}
with torch.no_grad():
    for B, H, W in ((1, 120, 160), (4, 120, 160)):
        enc = EdgeNextConvEncoder(128, expan_ratio=4, kernel_size=7, norm=None)
        synth.init_module_(enc, seed=5)
        enc = enc.to(dev).eval()
        x = torch.randn(B, 128, H, W, device=dev)
        y = torch.randn(B, 128, H, W, device=dev)
        pk1, b1 = update._packed(enc.pwconv1)
        pk2, b2 = update._packed(enc.pwconv2)
        out = torch.empty_like(y)
        fused = timed(lambda: ops.edgenext_mlp(x, y, pk1, b1, pk2, b2, gamma=enc.gamma, out=out))
        two = timed(lambda: update._conv(enc.pwconv2, [update._conv(enc.pwconv1, [x], "gelu")], gamma=enc.gamma,
                                         res=y))
        # phase stamps of one eager launch (100 MHz wall clock)
        nblk = B * ((H * W + 63) // 64)
        ts = torch.zeros(nblk * 8, dtype=torch.int64, device=dev)
        _lib.load().fsmi_debug_conv_timestamps(ts.data_ptr())
        ops.edgenext_mlp(x, y, pk1, b1, pk2, b2, gamma=enc.gamma, out=out)
        torch.cuda.synchronize()
        _lib.load().fsmi_debug_conv_timestamps(None)
        st = ts.view(nblk, 8).double().cpu() / 100.0       # us
        names = ["x_load+max", "split+gemm1", "gelu", "hmax_bar", "h_split", "gemm2", "epilogue"]
        ph = {n: round(float((st[:, k + 1] - st[:, k]).mean()), 2) for k, n in enumerate(names)}
        ph["block"] = round(float((st[:, 7] - st[:, 0]).mean()), 2)
        ph["span"] = round(float(st[:, 7].max() - st[:, 0].min()), 2)
        flops = 2 * 2 * 128 * 512 * B * H * W
        res[f"B{B}"] = {"fused_us": round(fused, 2), "two_conv_us": round(two, 2),
                        "fused_TFLOPs": round(flops / fused / 1e6, 1), "phases_us": ph}
print(json.dumps(res), flush=True)
