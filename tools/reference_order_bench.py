#!/usr/bin/env python3
"""Step time of the patched-reference call order (reference_order.forward_reference_order: unfused
volume, context after the volume path, one update_block call per iteration, MIOpen for the
reference's torch.nn convs) beside the fused FoundationStereo.forward, eager and hipGraph-replayed.

    python tools/reference_order_bench.py [--config cfg2] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from foundationstereo_amd import ops, synth  # noqa: E402
from tests.reference_order import forward_reference_order  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="cfg2")
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
dev = torch.device("cuda:0")
H, W, md, iters, vit, _ = bench.CONFIGS[a.config]
args = synth.make_args(max_disp=md, corr_levels=4, vit_size=vit)
model = bench.make_model(args, dev, 0)
fl, fr, vf = synth.backbone_features(1, H, W, vit, seed=0x5EED, shift_px=8)
model.feature.set_features([torch.from_numpy(x).to(dev) for x in fl], [torch.from_numpy(x).to(dev) for x in fr],
                           torch.from_numpy(vf).to(dev))
left, right = synth.stereo_images(1, H, W)
lt, rt = torch.from_numpy(left).to(dev), torch.from_numpy(right).to(dev)


def timed(fn):
    with torch.no_grad():
        fn()
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            out = fn()
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / a.reps * 1e3, out


res = {"config": a.config, "iters": iters}
res["reference_order_ms"], out_ref = timed(lambda: forward_reference_order(model, lt, rt, iters=iters, test_mode=True))
res["fused_eager_ms"], out_fused = timed(lambda: model(lt, rt, iters=iters, test_mode=True))
with torch.no_grad():
    gr = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(gr):
        out_g = model(lt, rt, iters=iters, test_mode=True)
res["fused_graph_ms"], _ = timed(lambda: (gr.replay(), out_g)[1])
res["max_abs_diff_px"] = float((out_ref - out_fused).abs().max())
ops.check_range()
print(json.dumps(res))
