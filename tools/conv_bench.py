#!/usr/bin/env python3
"""fsmi_conv2d (fp32 MFMA implicit GEMM) vs MIOpen (torch F.conv2d) on the refinement-loop layer shapes.

    python tools/conv_bench.py [--reps 20]
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
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--all-cfg", action="store_true")
ap.add_argument("--mode", default="x3", choices=["x3", "f32", "halo"])
ap.add_argument("--cfg", type=int, default=-1, help="tile config for the main timing (-1 auto)")
ap.add_argument("--only", default="", help="comma-separated layer names")
ap.add_argument("--no-miopen", action="store_true")
ap.add_argument("--nsplit", type=int, nargs="*", default=[], help="halo: also time these split-K factors")
a = ap.parse_args()
dev = torch.device("cuda:0")
torch.backends.cudnn.benchmark = False

# (name, cin, cout, k, H, W) at cfg2 (1/4 = 120x160, 1/8 = 60x80, 1/16 = 30x40)
SHAPES = [
    ("gru04.conv0", 384, 384, 3, 120, 160), ("gru04.conv1", 512, 512, 3, 120, 160),
    ("gru04.zr_l", 512, 256, 3, 120, 160), ("gru04.zr_s", 512, 256, 1, 120, 160),
    ("gru04.q_l", 512, 128, 3, 120, 160), ("gru04.q_s", 512, 128, 1, 120, 160),
    ("enc.convc1", 1044, 256, 1, 120, 160), ("enc.convc2", 256, 256, 3, 120, 160),
    ("enc.convd1", 1, 64, 7, 120, 160), ("enc.convd2", 64, 64, 3, 120, 160), ("enc.conv", 320, 127, 3, 120, 160),
    ("head.conv", 128, 128, 3, 120, 160), ("head.pw1", 128, 512, 1, 120, 160), ("head.pw2", 512, 128, 1, 120, 160),
    ("head.out", 128, 1, 3, 120, 160), ("mask.0", 128, 64, 3, 120, 160), ("mask.2", 64, 32, 3, 120, 160),
    ("gru08.conv0", 384, 384, 3, 60, 80), ("gru08.conv1", 512, 512, 3, 60, 80), ("gru08.zr_l", 512, 256, 3, 60, 80),
    ("gru08.zr_s", 512, 256, 1, 60, 80), ("gru08.q_l", 512, 128, 3, 60, 80), ("gru08.q_s", 512, 128, 1, 60, 80),
    ("gru16.conv0", 256, 256, 3, 30, 40), ("gru16.conv1", 384, 384, 3, 30, 40), ("gru16.zr_l", 384, 256, 3, 30, 40),
    ("gru16.zr_s", 384, 256, 1, 30, 40), ("gru16.q_l", 384, 128, 3, 30, 40), ("gru16.q_s", 384, 128, 1, 30, 40),
]


def timeit(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / a.reps


rows = []
tot_m = tot_f = 0.0
for name, cin, cout, k, H, W in SHAPES:
    if a.mode == "halo" and k not in (1, 3):
        continue
    if a.only and name not in a.only.split(","):
        continue
    x = torch.randn(1, cin, H, W, device=dev)
    w = torch.randn(cout, cin, k, k, device=dev) * 0.05
    b = torch.randn(cout, device=dev)
    pk = ops.PackedConv(w, mode=a.mode)
    fl = 2.0 * cin * cout * k * k * H * W
    t_m = 1.0 if a.no_miopen else timeit(lambda: F.relu(F.conv2d(x, w, b, padding=k // 2)))
    t_f = timeit(lambda: ops.conv2d([x], pk, bias=b, act="relu", cfg=a.cfg))
    row = {"layer": name, "miopen_us": round(t_m, 1), "fsmi_us": round(t_f, 1),
           "fsmi_TF": round(fl / t_f / 1e6, 1), "speedup": round(t_m / t_f, 2)}
    for ns in a.nsplit:
        row[f"split{ns}_us"] = round(timeit(lambda: ops.conv2d([x], pk, bias=b, act="relu", nsplit=ns)), 1)
    if a.all_cfg:
        for c in range(6 if a.mode == "halo" else 4):
            row[f"cfg{c}_us"] = round(timeit(lambda: ops.conv2d([x], pk, bias=b, act="relu", cfg=c)), 1)
    rows.append(row)
    tot_m += t_m
    tot_f += t_f
    print(json.dumps(row), flush=True)
print(json.dumps({"total_miopen_us": round(tot_m, 1), "total_fsmi_us": round(tot_f, 1)}))
