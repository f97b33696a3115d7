#!/usr/bin/env python3
"""Which layers of one eager forward still reach torch / MIOpen convolutions (and InstanceNorm /
interpolate): every module whose forward calls F.conv2d / conv_transpose2d / instance_norm is named
with its input shape (forward hooks + a patched functional).  The rest of the forward is HIP.

    python tools/torch_conv_census.py [--config cfg2] [--with-backbone] [--out profiles/r06_torch_conv_census.txt]
"""
import argparse
import collections
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import bench  # noqa: E402
from foundationstereo_amd import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="cfg2")
ap.add_argument("--with-backbone", action="store_true")
ap.add_argument("--out", default="")
a = ap.parse_args()
dev = torch.device("cuda:0")
H, W, md, iters, vit, per = bench.CONFIGS[a.config]
args = synth.make_args(max_disp=md, corr_levels=4, vit_size=vit)
if a.with_backbone:
    args["backbone"] = "real"
model = bench.make_model(args, dev, 0)
if not a.with_backbone:
    fl, fr, vf = synth.backbone_features(1, H, W, vit, seed=0x5EED, shift_px=8)
    model.feature.set_features([torch.from_numpy(x).to(dev) for x in fl], [torch.from_numpy(x).to(dev) for x in fr],
                               torch.from_numpy(vf).to(dev), size=(H, W))
left, right = synth.stereo_images(1, H, W)
L, R = torch.from_numpy(left).to(dev), torch.from_numpy(right).to(dev)
with torch.no_grad():
    model(L, R, iters=iters, test_mode=True)          # warm: weight packing, caches
torch.cuda.synchronize()

stack = []
calls = collections.Counter()


def pre(mod, inp):
    stack.append(mod)


def post(mod, inp, out):
    stack.pop()


names = {m: n for n, m in model.named_modules()}
hooks = [m.register_forward_pre_hook(pre) for m in model.modules()] + [m.register_forward_hook(post)
                                                                      for m in model.modules()]


def wrap(fn_name):
    orig = getattr(F, fn_name)

    def f(x, *args, **kw):
        owner = next((names[m] for m in reversed(stack) if m in names), "?")
        calls[(fn_name, owner or "<model>", tuple(x.shape))] += 1
        return orig(x, *args, **kw)
    setattr(F, fn_name, f)


for fn in ("conv2d", "conv_transpose2d", "conv3d", "instance_norm", "interpolate", "scaled_dot_product_attention"):
    wrap(fn)
with torch.no_grad():
    model(L, R, iters=iters, test_mode=True)
torch.cuda.synchronize()
lines = [f"{a.config}{' with backbone' if a.with_backbone else ''}: torch functional calls in one eager forward "
         f"(fn, owning module, input shape, count)"]
for (fn, owner, shp), n in sorted(calls.items()):
    lines.append(f"  {fn:28s} {owner:40s} {str(shp):28s} x{n}")
print("\n".join(lines))
if a.out:
    with open(a.out, "w") as f:
        f.write("\n".join(lines) + "\n")
