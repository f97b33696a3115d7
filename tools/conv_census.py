#!/usr/bin/env python3
"""Per-shape conv census of one forward: call counts x the tuned per-call time (tuning table),
sorted by total -- where the conv time of a workload goes.  GPU box:

    python tools/conv_census.py [--config cfg2] [--iters 32]
"""
import argparse
import json
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from foundationstereo_amd import ops, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="cfg2")
ap.add_argument("--iters", type=int, default=None)
a = ap.parse_args()
dev = torch.device("cuda:0")
H, W, md, iters, vit, per_gpu = bench.CONFIGS[a.config]
iters = a.iters or iters
args = synth.make_args(max_disp=md, corr_levels=4, vit_size=vit)
model = bench.make_model(args, dev, 0)
for (ph, pw) in bench.pass_sizes(a.config, H, W):
    feats = [synth.backbone_features(1, ph, pw, vit, seed=0x5EED + i, shift_px=8) for i in range(per_gpu)]
    fl = [torch.from_numpy(np.concatenate([f[0][j] for f in feats])).to(dev) for j in range(4)]
    fr = [torch.from_numpy(np.concatenate([f[1][j] for f in feats])).to(dev) for j in range(4)]
    vf = torch.from_numpy(np.concatenate([f[2] for f in feats])).to(dev)
    model.feature.set_features(fl, fr, vf, size=(ph, pw))
left, right = synth.stereo_images(per_gpu, H, W)
lt, rt = torch.from_numpy(left).to(dev), torch.from_numpy(right).to(dev)
ops._RECORD = {}
with torch.no_grad():
    if a.config in bench.HIERA:
        model.run_hierachical(lt, rt, iters=iters, test_mode=True)
    else:
        model(lt, rt, iters=iters, test_mode=True)
torch.cuda.synchronize()
counts, ops._RECORD = ops._RECORD, None
db = json.load(open(ops._TUNE_PATH))["entries"]
rows, tot, totf = [], 0.0, 0.0
for k, n in counts.items():
    ks, kd, cin, cout, B, D, Hh, Ww = (int(v) for v in re.findall(r"\d+", k))
    e = db.get(k, {})
    us = e.get("us", float("nan"))
    fl = 2.0 * cin * cout * ks * ks * kd * B * D * Hh * Ww
    rows.append((n * us, n, us, fl / us / 1e6 if us == us else 0, e.get("cfg"), e.get("nsplit"), k))
    tot += n * us if us == us else 0
    totf += n * fl
rows.sort(reverse=True)
for r in rows:
    print(f"{r[0] / 1e3:8.2f} ms  {r[1]:4d} x {r[2]:7.1f} us  {r[3]:6.1f} TF/s  cfg {r[4]} s {r[5]}  {r[6]}")
print(json.dumps({"config": a.config, "iters": iters, "conv_ms": round(tot / 1e3, 2), "conv_tflop": round(totf / 1e12, 3),
                  "tflops": round(totf / tot / 1e6, 1)}))
