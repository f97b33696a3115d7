#!/usr/bin/env python3
"""Diagnostic: repeat the pointwise-tile range case (tests/test_gpu_parity.py::test_conv2d_pw_range) and
report, per (cfg, scale, nsplit), the worst relative error over the repetitions and where the worst
element sits (b, co, pixel), to tell a deterministic fault from an intermittent one."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from foundationstereo_amd import _lib, ops, synth  # noqa: E402

_lib.load()
dev = torch.device("cuda:0")
reps = int(os.environ.get("REPS", "20"))
B, H, W, cin, cout = 1, 16, 40, 96, 130
for scale in (3e5, 1e3, 1e-4, 1e-7):
    x = torch.from_numpy(synth.normal(391, (B, cin, H, W)) * scale)
    w = torch.from_numpy(synth.normal(392, (cout, cin, 1, 1), 0.2))
    ref = F.conv2d(x.double(), w.double())
    pk = ops.PackedConv(w.float().to(dev), mode="halo")
    xg = x.float().to(dev)
    for cfg in (24, 25, 26, 27, 28, 29):
        for nsplit in (1, 2, 3):
            worst, where, bad = 0.0, None, 0
            for _ in range(reps):
                out = ops.conv2d([xg], pk, cfg=cfg, nsplit=nsplit).double().cpu()
                d = (out - ref).abs() / ref.abs().max()
                e = float(d.max())
                if e > 3e-6:
                    bad += 1
                if e > worst:
                    worst = e
                    idx = int(d.argmax())
                    where = (idx // (cout * H * W), (idx // (H * W)) % cout, idx % (H * W))
            print(f"scale {scale:g} cfg {cfg} nsplit {nsplit}: worst {worst:.2e} at {where}, bad {bad}/{reps}",
                  flush=True)
print("overflow flag:", ops.range_overflowed(reset=True))
