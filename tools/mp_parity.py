#!/usr/bin/env python3
"""Parity and speed of the conv precision modes at a full workload vs the CPU oracle.

    python tools/mp_parity.py [--config cfg2] [--iters 32]

Runs the product forward in fp32, fp16-autocast and bf16-autocast (dense
convs only; volumes, lookup and gates stay fp32) and the fp32 CPU oracle on
the same inputs; prints max |dd| (px) and ms per forward for each mode.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import oracle  # noqa: E402
from foundationstereo_amd import synth  # noqa: E402
from foundationstereo_amd.foundation_stereo import FoundationStereo  # noqa: E402

CFG = {"cfg1": (256, 320, 64, "vits"), "cfg2": (480, 640, 192, "vits"), "cfg4": (384, 1248, 256, "vitl")}

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="cfg2")
ap.add_argument("--iters", type=int, default=32)
ap.add_argument("--levels", type=int, default=4)
a = ap.parse_args()
H, W, md, vit = CFG[a.config]
dev = torch.device("cuda:0")
T = torch.from_numpy
fl, fr, vf = synth.backbone_features(1, H, W, vit, shift_px=8)
left, right = synth.stereo_images(1, H, W)
res = {}
base = synth.make_args(max_disp=md, corr_levels=a.levels, vit_size=vit)
m = FoundationStereo(base).eval()
synth.init_module_(m, seed=1234)
P = {k: v.clone() for k, v in m.state_dict().items()}
m = m.to(dev)
m.feature.set_features([T(x).to(dev) for x in fl], [T(x).to(dev) for x in fr], T(vf).to(dev))
outs = {}
for mode in ("fp32", "float16", "bfloat16"):
    m.args["mixed_precision"] = mode != "fp32"
    m.args["mixed_dtype"] = "float16" if mode == "fp32" else mode
    with torch.no_grad():
        for _ in range(2):
            out = m(T(left).to(dev), T(right).to(dev), iters=a.iters, test_mode=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            out = m(T(left).to(dev), T(right).to(dev), iters=a.iters, test_mode=True)
        torch.cuda.synchronize()
    outs[mode] = out.float().cpu()
    res[mode] = {"ms": (time.perf_counter() - t0) / 3 * 1e3}
torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", 16)))
with torch.no_grad():
    ref = oracle.oracle_forward(P, base, T(left), T(right), [T(x) for x in fl], [T(x) for x in fr], T(vf),
                                iters=a.iters)
for mode, o in outs.items():
    d = (o - ref).abs()
    res[mode].update(max_abs_px=float(d.max()), mean_abs_px=float(d.mean()), p99_px=float(d.flatten().kthvalue(
        int(0.99 * d.numel())).values))
print(json.dumps({"config": a.config, "iters": a.iters, "levels": a.levels, "modes": res}))
