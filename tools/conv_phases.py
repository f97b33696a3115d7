#!/usr/bin/env python3
"""Per-block timeline of one halo conv (fsmi_debug_conv_timestamps): block start spread (rounds),
per-chunk staging-to-staging durations, epilogue, and the resulting MFMA-issue fraction.

    python tools/conv_phases.py --layer gru04.conv1 [--cfg 3 --nsplit 2]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
from foundationstereo_amd import _lib, ops  # noqa: E402

SHAPES = {"gru04.conv0": (384, 384, 3, 120, 160), "gru04.conv1": (512, 512, 3, 120, 160),
          "gru04.zr_l": (512, 256, 3, 120, 160), "gru04.zr_s": (512, 256, 1, 120, 160),
          "gru04.q_l": (512, 128, 3, 120, 160), "enc.convc1": (1044, 256, 1, 120, 160),
          "enc.convc2": (256, 256, 3, 120, 160), "gru08.conv1": (512, 512, 3, 60, 80),
          "head.pw1": (128, 512, 1, 120, 160), "head.pw2": (512, 128, 1, 120, 160)}
ap = argparse.ArgumentParser()
ap.add_argument("--layer", default="gru04.conv1")
ap.add_argument("--cfg", type=int, default=-1)
ap.add_argument("--nsplit", type=int, default=-1)
a = ap.parse_args()
cin, cout, k, H, W = SHAPES[a.layer]
dev = torch.device("cuda:0")
x = torch.randn(1, cin, H, W, device=dev)
w = torch.randn(cout, cin, k, k, device=dev) * 0.05
b = torch.randn(cout, device=dev)
pk = ops.PackedConv(w, mode="halo")
run = lambda: ops.conv2d([x], pk, bias=b, act="relu", cfg=a.cfg, nsplit=a.nsplit)  # noqa: E731
for _ in range(3):
    run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    run()
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1e3 / 20
buf = torch.zeros(40 * 65536, dtype=torch.int64, device=dev)
lib = _lib.load()
lib.fsmi_debug_conv_timestamps(buf.data_ptr())
run()
torch.cuda.synchronize()
lib.fsmi_debug_conv_timestamps(None)
t = buf.view(-1, 40).cpu()
used = t[:, 39] != 0
t = t[used]
nblk = t.shape[0]
nch = int((t[0, 39] >> 32).item())
ts = t[:, :39].double() / 100.0
t0 = ts[:, 0].min()
ts = ts - t0
start, end = ts[:, 0], ts[:, 38]
span = float(end.max())
flops = 2 * cin * cout * k * k * H * W
print(f"{a.layer} cfg {a.cfg} nsplit {a.nsplit}: {us:.1f} us/launch ({flops / us / 1e6:.0f} TF/s fp32-eq), "
      f"{nblk} blocks, {nch} chunks/block, stamped span {span:.1f} us")
srt = start.sort().values
print("  block start quantiles (us): " + " ".join(f"{q:.2f}:{float(srt[int(q * (nblk - 1))]):.1f}"
                                              for q in (0.0, 0.25, 0.5, 0.6, 0.75, 0.9, 1.0)))
life = end - start
print(f"  block lifetime: median {float(life.median()):.2f}  min {float(life.min()):.2f}  max {float(life.max()):.2f} us")
pro = ts[:, 1] - ts[:, 0]
print(f"  prologue (start -> first staging): median {float(pro.median()):.2f} us")
if nch > 1:
    ch = ts[:, 2:1 + nch] - ts[:, 1:nch]
    print(f"  chunk (staging -> staging): median {float(ch.median()):.2f}  p10 {float(ch.quantile(0.1)):.2f}  "
          f"p90 {float(ch.quantile(0.9)):.2f} us")
last = ts[:, 37] - ts[:, nch]
epi = ts[:, 38] - ts[:, 37]
print(f"  last chunk: median {float(last.median()):.2f} us   epilogue: median {float(epi.median()):.2f}  "
      f"p90 {float(epi.quantile(0.9)):.2f} us")
