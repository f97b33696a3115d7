#!/usr/bin/env python3
"""Python call sites of torch conv2d / copy_ / add / relu during one eager cfg2 forward (which ATen
launches remain in the hot path).  GPU box: python tools/call_sites.py"""
import collections
import os
import sys
import traceback

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import bench  # noqa: E402
from foundationstereo_amd import synth  # noqa: E402

dev = torch.device("cuda:0")
H, W, md, iters, vit, per_gpu = bench.CONFIGS["cfg2"]
args = synth.make_args(max_disp=md, corr_levels=4, vit_size=vit)
model = bench.make_model(args, dev, 0)
f0 = synth.backbone_features(1, H, W, vit, seed=0x5EED, shift_px=8)
model.feature.set_features([torch.from_numpy(f0[0][j]).to(dev) for j in range(4)],
                           [torch.from_numpy(f0[1][j]).to(dev) for j in range(4)],
                           torch.from_numpy(f0[2]).to(dev), size=(H, W))
left, right = synth.stereo_images(1, H, W)
lt, rt = torch.from_numpy(left).to(dev), torch.from_numpy(right).to(dev)
sites = collections.Counter()


def site():
    st = [f for f in traceback.extract_stack()[:-2] if "foundationstereo_amd" in f.filename]
    return " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in st[-3:][::-1])


def wrap(obj, name):
    orig = getattr(obj, name)

    def w(*a, **k):
        sites[(name, site())] += 1
        return orig(*a, **k)
    setattr(obj, name, w)


with torch.no_grad():
    for _ in range(2):
        model(lt, rt, iters=iters, test_mode=True)
    for obj, name in ((F, "conv2d"), (torch.Tensor, "copy_"), (torch.Tensor, "__add__"), (torch, "relu"),
                      (F, "relu"), (torch.Tensor, "add_"), (torch, "cat"), (torch, "sigmoid"),
                      (torch.Tensor, "__mul__"), (F, "leaky_relu"), (F, "batch_norm"), (F, "conv3d"),
                      (F, "conv_transpose3d"), (torch, "tanh"), (F, "instance_norm")):
        wrap(obj, name)
    torch.nn.modules.conv.Conv2d._conv_forward.__globals__["F"] = F
    model(lt, rt, iters=iters, test_mode=True)
    torch.cuda.synchronize()
for (name, s), n in sorted(sites.items(), key=lambda x: -x[1]):
    print(f"{n:4d} {name:18s} {s}")
