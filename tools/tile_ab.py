#!/usr/bin/env python3
"""A/B of conv tile configurations per layer shape, timed inside a replayed hipGraph (no host
launch overhead), with each candidate checked against fp64 torch.

    python tools/tile_ab.py [--set loop|depth|all] [--cfgs 9,41,...] [--reps 20]

* loop: the cfg2 refinement-loop 2D layers (tools/conv_bench.py SHAPES), each at its tuned
  (cfg, nsplit) and at the pipelined variant of the same tile (cfg 32 + c, conv_halo_pipe_kernel);
* depth: the hourglass (17, 1, 1) convs at cfg2 on the depth-blocked tile (cfg 30) vs the generic
  volume tiles.
Prints one JSON line per (layer, cfg): us per launch, TFLOP/s (fp32-equivalent), max rel err.
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
ap.add_argument("--set", default="all")
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--only", default="")
a = ap.parse_args()
dev = torch.device("cuda:0")

LOOP = [("gru04.conv0", 384, 384, 3, 120, 160), ("gru04.conv1", 512, 512, 3, 120, 160),
        ("gru04.zr_l", 512, 256, 3, 120, 160), ("gru04.q_l", 512, 128, 3, 120, 160),
        ("enc.convc2", 256, 256, 3, 120, 160), ("enc.conv", 320, 127, 3, 120, 160),
        ("head.conv", 128, 128, 3, 120, 160), ("enc.convd2", 64, 64, 3, 120, 160),
        ("gru04.zr_s", 512, 256, 1, 120, 160), ("gru04.q_s", 512, 128, 1, 120, 160),
        ("enc.convc1", 1044, 256, 1, 120, 160), ("head.pw1", 128, 512, 1, 120, 160), ("head.pw2", 512, 128, 1, 120, 160),
        ("gru08.conv0", 384, 384, 3, 60, 80), ("gru08.conv1", 512, 512, 3, 60, 80),
        ("gru08.zr_l", 512, 256, 3, 60, 80), ("gru08.q_l", 512, 128, 3, 60, 80),
        ("gru16.conv1", 384, 384, 3, 30, 40), ("gru16.zr_l", 384, 256, 3, 30, 40)]
# (name, C, D, H, W): Conv3dNormActReduced.conv2 at cfg2 (D4 = 48 at 120 x 160)
DEPTH = [("conv_out", 28, 48, 120, 160), ("agg_1", 56, 24, 60, 80), ("agg_0", 112, 12, 30, 40),
         ("conv3", 168, 6, 15, 20)]
# (name, cin, cout, kd, k, D, H, W): the volume convs of corr_stem / classifier / Conv3dNormActReduced.conv1
VOL = [("stem3x3x3", 28, 28, 3, 3, 48, 120, 160), ("cls3x3x3", 28, 14, 3, 3, 48, 120, 160),
       ("cls14", 14, 14, 3, 3, 48, 120, 160), ("red1x3x3", 28, 28, 1, 3, 48, 120, 160),
       ("agg1_1x3x3", 56, 56, 1, 3, 24, 60, 80)]


def graph_time(fn):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(a.reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e30
    for _ in range(5):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / a.reps)
    return best


def rel(out, ref):
    return float((out.double() - ref).abs().max() / ref.abs().max())


rows = []
if a.set in ("loop", "all"):
    for name, cin, cout, k, H, W in LOOP:
        if a.only and name not in a.only.split(","):
            continue
        gen = torch.Generator(device="cpu").manual_seed(cin + cout)
        x = torch.randn(1, cin, H, W, generator=gen).to(dev)
        w = (torch.randn(cout, cin, k, k, generator=gen) * 0.05).to(dev)
        b = torch.randn(cout, generator=gen).to(dev)
        pk = ops.PackedConv(w, mode="halo")
        ref = F.relu(F.conv2d(x.double(), w.double(), b.double(), padding=k // 2))
        tcfg, tns = ops._tuned(k, 1, cin, cout, 1, 1, H, W, -1, -1)
        cands = [(tcfg, tns)]
        if 2 <= tcfg <= 9:
            cands.append((tcfg + 32, tns))
        elif tcfg >= 16:
            for c in (3, 4, 9):
                cands += [(c, tns), (c + 32, tns)]
        if k == 1:
            cands += [(c, ns) for c in (24, 25, 26, 27, 28, 29) for ns in (1, 2, 3) if (c, ns) != (tcfg, tns)]
        fl = 2.0 * cin * cout * k * k * H * W
        for cfg, ns in cands:
            fn = lambda: ops.conv2d([x], pk, bias=b, act="relu", cfg=cfg, nsplit=ns)  # noqa: E731
            us = graph_time(fn)
            r = {"layer": name, "cfg": cfg, "nsplit": ns, "us": round(us, 2), "TF": round(fl / us / 1e6, 1),
                 "rel_err": rel(fn(), ref)}
            rows.append(r)
            print(json.dumps(r), flush=True)
if a.set in ("depth", "all"):
    for name, C, D, H, W in DEPTH:
        if a.only and name not in a.only.split(","):
            continue
        gen = torch.Generator(device="cpu").manual_seed(C + D)
        x = torch.randn(1, C, D, H, W, generator=gen).to(dev)
        w = (torch.randn(C, C, 17, 1, 1, generator=gen) * 0.05).to(dev)
        b = torch.randn(C, generator=gen).to(dev)
        pk = ops.PackedConv(w, mode="halo")
        ref = F.relu(F.conv3d(x.double(), w.double(), b.double(), padding=(8, 0, 0)))
        tcfg, tns = ops._tuned(1, 17, C, C, 1, D, H, W, -1, -1)
        fl = 2.0 * C * C * 17 * D * H * W
        for cfg, ns in [(30, 1), (tcfg, tns), (7, 1), (4, 1)]:
            fn = lambda: ops.conv3d(x, pk, bias=b, act="relu", cfg=cfg, nsplit=ns)  # noqa: E731
            us = graph_time(fn)
            r = {"layer": name, "cfg": cfg, "nsplit": ns, "us": round(us, 2), "TF": round(fl / us / 1e6, 1),
                 "rel_err": rel(fn(), ref)}
            rows.append(r)
            print(json.dumps(r), flush=True)
if a.set in ("vol", "all"):
    for name, cin, cout, kd, k, D, H, W in VOL:
        if a.only and name not in a.only.split(","):
            continue
        gen = torch.Generator(device="cpu").manual_seed(cin + cout + kd)
        x = torch.randn(1, cin, D, H, W, generator=gen).to(dev)
        w = (torch.randn(cout, cin, kd, k, k, generator=gen) * 0.05).to(dev)
        b = torch.randn(cout, generator=gen).to(dev)
        pk = ops.PackedConv(w, mode="halo")
        ref = F.relu(F.conv3d(x.double(), w.double(), b.double(), padding=(kd // 2, k // 2, k // 2)))
        tcfg, tns = ops._tuned(k, kd, cin, cout, 1, D, H, W, -1, -1)
        fl = 2.0 * cin * cout * kd * k * k * D * H * W
        for cfg, ns in [(tcfg, tns), (7, 1), (6, 1), (5, 1), (23, 1)]:
            fn = lambda: ops.conv3d(x, pk, bias=b, act="relu", cfg=cfg, nsplit=ns)  # noqa: E731
            us = graph_time(fn)
            r = {"layer": name, "cfg": cfg, "nsplit": ns, "us": round(us, 2), "TF": round(fl / us / 1e6, 1),
                 "rel_err": rel(fn(), ref)}
            rows.append(r)
            print(json.dumps(r), flush=True)
if a.set in ("cls", "all"):
    # the classifier head Conv3d(14, 1, 7) (fp32 FMA direct kernel) at cfg2 / cfg3-per-GPU
    for name, B, D, H, W in [("cls7_cfg2", 1, 48, 120, 160), ("cls7_b4", 4, 48, 120, 160)]:
        gen = torch.Generator(device="cpu").manual_seed(7)
        x = torch.randn(B, 14, D, H, W, generator=gen).to(dev)
        w = (torch.randn(1, 14, 7, 7, 7, generator=gen) * 0.05).to(dev)
        b = torch.randn(1, generator=gen).to(dev)
        ref = F.conv3d(x.double(), w.double(), b.double(), padding=3)
        fl = 2.0 * 14 * 343 * B * D * H * W
        fn = lambda: ops.conv3d_direct(x, w, b)  # noqa: E731
        us = graph_time(fn)
        r = {"layer": name, "us": round(us, 2), "TF": round(fl / us / 1e6, 1), "rel_err": rel(fn(), ref)}
        print(json.dumps(r), flush=True)
ops.range_overflowed(reset=True)
