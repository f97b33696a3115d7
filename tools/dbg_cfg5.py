#!/usr/bin/env python3
"""Diagnostics for the cfg5 hierarchical run: saves the product's coarse-pass and final
disparities (and the range flag) to gpurun_out/dbg_cfg5_<tag>.npz; with --oracle also the oracle's."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from foundationstereo_amd import ops, synth  # noqa: E402
from foundationstereo_amd.foundation_stereo import FoundationStereo  # noqa: E402

tag = sys.argv[1]
H, W, md, iters = (int(v) for v in os.environ.get("DBG_SHAPE", "1024,1536,320,22").split(","))
args = synth.make_args(max_disp=md, corr_levels=4, vit_size="vitl")
m = FoundationStereo(args).eval()
synth.init_module_(m, seed=1234)
m = m.cuda()
m.feature.shift_px = 8
left, right = synth.stereo_images(1, H, W)
cap = []
orig = FoundationStereo.forward


def fwd(self, *a, **k):
    out = orig(self, *a, **k)
    cap.append(out.detach().float().cpu().numpy())
    return out


FoundationStereo.forward = fwd
ops.range_overflowed(reset=True)
with torch.no_grad():
    out = m.run_hierachical(torch.from_numpy(left).cuda(), torch.from_numpy(right).cuda(), iters=iters,
                            test_mode=True).cpu().numpy()
flag = ops.range_overflowed(reset=True)
res = {"out": out, "small": cap[0], "flag": np.array(flag)}
if "--oracle" in sys.argv:
    import oracle
    P = {k: v.cpu() for k, v in m.state_dict().items()}

    def features(B, h, w):
        fl, fr, vf = synth.backbone_features(B, h, w, "vitl", shift_px=8)
        return [torch.from_numpy(x) for x in fl], [torch.from_numpy(x) for x in fr], torch.from_numpy(vf)
    with torch.no_grad():
        ref, aux = oracle.oracle_hierarchical(P, args, torch.from_numpy(left), torch.from_numpy(right), features,
                                              iters=iters, return_aux=True)
    res["ref"] = ref.numpy()
    res["ref_small"] = aux["disp_small"].numpy()
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
np.savez_compressed(os.path.join(REPO, "gpurun_out", f"dbg_cfg5_{tag}.npz"), **res)
print(tag, "flag", flag, "out mean", float(out.mean()))
