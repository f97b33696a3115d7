#!/usr/bin/env python3
"""Attribute the non-fsmi (ATen) launches of one eager cfg2 forward to their Python call sites.
GPU box: python tools/torch_prof.py"""
import collections
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import bench  # noqa: E402
from foundationstereo_amd import synth  # noqa: E402

dev = torch.device("cuda:0")
H, W, md, iters, vit, per_gpu = bench.CONFIGS["cfg2"]
args = synth.make_args(max_disp=md, corr_levels=4, vit_size=vit)
model = bench.make_model(args, dev, 0)
feats = [synth.backbone_features(1, H, W, vit, seed=0x5EED, shift_px=8)]
model.feature.set_features([torch.from_numpy(feats[0][0][j]).to(dev) for j in range(4)],
                           [torch.from_numpy(feats[0][1][j]).to(dev) for j in range(4)],
                           torch.from_numpy(feats[0][2]).to(dev), size=(H, W))
left, right = synth.stereo_images(1, H, W)
lt, rt = torch.from_numpy(left).to(dev), torch.from_numpy(right).to(dev)
with torch.no_grad():
    for _ in range(2):
        model(lt, rt, iters=iters, test_mode=True)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
        model(lt, rt, iters=iters, test_mode=True)
        torch.cuda.synchronize()
for ka in prof.key_averages(group_by_stack_n=12):
    if ka.key not in ("aten::conv2d", "aten::copy_", "aten::add", "aten::relu", "aten::relu_", "aten::batch_norm",
                      "aten::add_", "aten::cat", "aten::sigmoid", "aten::mul", "aten::new_empty"):
        continue
    st = [f for f in ka.stack if "foundationstereo_amd" in f or "bench.py" in f][:3]
    print(f"{ka.count:5d}  {ka.key:20s} " + " <- ".join(x.split("repo/")[-1] for x in st))
