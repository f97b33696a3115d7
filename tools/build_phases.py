#!/usr/bin/env python3
"""Per-block phase timeline of the single-pass build (FSMI_BUILD_DBG=4: thread 0 of every block
records wall_clock64() at start, after each group barrier, after the epilogue staging, after
its stores issue and after they drain).  Prints median / p90 phase durations in us and the
spread of block start / end times.

    python tools/build_phases.py [--config cfg2] [--tile 8,12]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
from foundationstereo_amd import ops  # noqa: E402

CFG = {"cfg2": (480, 640, 192, 128), "cfg2l": (480, 640, 192, 224), "cfg5": (1024, 1536, 320, 224)}
ap = argparse.ArgumentParser()
ap.add_argument("--config", default="cfg2")
ap.add_argument("--tile", default="")
a = ap.parse_args()
H, W, md, C = CFG[a.config]
H4, W4, D4 = H // 4, W // 4, md // 4
dev = torch.device("cuda:0")
fl = torch.randn(1, C, H4, W4, device=dev)
fr = torch.randn(1, C, H4, W4, device=dev)
A = torch.randn(1, 28, H4, W4, device=dev)
Bm = torch.randn(1, 28, H4, W4, device=dev)
Wg = torch.randn(28, 8, device=dev)
os.environ["FSMI_BUILD_TILE"] = a.tile
for _ in range(3):
    ops.comb_volume_stem(fl, fr, A, Bm, Wg, D4)
os.environ["FSMI_BUILD_DBG"] = "4"
out = ops.comb_volume_stem(fl, fr, A, Bm, Wg, D4)
torch.cuda.synchronize()
raw = out.view(-1).view(torch.int64)
WQ, DQN = (int(v) for v in a.tile.split(",")) if a.tile else (20, 12)
nblk = H4 * ((W4 + 4 * WQ - 1) // (4 * WQ)) * ((D4 + 4 * DQN - 1) // (4 * DQN))
ts = raw[: nblk * 16].view(nblk, 16)[:, :12].double().cpu() / 100.0   # 100 MHz ticks -> us
t0 = ts[:, 0].min()
ts = ts - t0
names = ["start"] + [f"g{g}" for g in range(8)] + ["stage", "issued", "drained"]
print(f"{a.config} tile {a.tile or 'auto'}: {nblk} blocks, kernel span {float(ts[:, 11].max()):.1f} us")
print(f"  block start: median {float(ts[:, 0].median()):.2f}  max {float(ts[:, 0].max()):.2f} us")
for k in range(1, 12):
    d = ts[:, k] - ts[:, k - 1]
    print(f"  {names[k - 1]:>7} -> {names[k]:<7}  median {float(d.median()):6.2f}  p90 {float(d.quantile(0.9)):6.2f} us")
