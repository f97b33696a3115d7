"""The one-round 80-pixel EdgeNeXt MLP tile (csrc/edgenext_mlp.hip edgenext_mlp80_kernel, opt-in with
FSMI_MLP_PX=80: 16x16x32 MFMA fragments, the hidden map in two halves with their own exponents) vs
fp64 torch.  The tile is chosen once per process, so the check runs in a child process with the knob
set; the child also confirms the 80-pixel launch ran (its phase stamps cover 80-pixel blocks)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, os, sys
sys.path.insert(0, os.environ["REPO"])
import numpy as np, torch
from foundationstereo_amd import _lib, ops, synth, update
from foundationstereo_amd.submodule import EdgeNextConvEncoder
dev = torch.device("cuda:0")
_lib.load()
res = {}
for B, H, W, gscale in ((1, 120, 160, 1.0), (2, 7, 13, 1.0), (1, 1, 1, 1.0), (1, 24, 24, 1e-6)):
    C = 128
    enc = EdgeNextConvEncoder(C, expan_ratio=4, kernel_size=7, norm=None)
    synth.init_module_(enc, seed=211)
    with torch.no_grad():
        enc.gamma.copy_(torch.from_numpy(synth.uniform(212, (C,), 0.5, 1.5)) * gscale)
    enc = enc.to(dev).eval()
    x = synth.normal(213, (B, C, H, W), 1.5)
    y = synth.normal(214, (B, C, H, W))
    pk1, b1 = update._packed(enc.pwconv1)
    pk2, b2 = update._packed(enc.pwconv2)
    nblk = B * ((H * W + 79) // 80)
    ts = torch.zeros(nblk * 8 + 64, dtype=torch.int64, device=dev)
    _lib.load().fsmi_debug_conv_timestamps(ts.data_ptr())
    with torch.no_grad():
        out = ops.edgenext_mlp(torch.from_numpy(x).to(dev), torch.from_numpy(y).to(dev), pk1, b1, pk2, b2,
                               gamma=enc.gamma)
    torch.cuda.synchronize()
    _lib.load().fsmi_debug_conv_timestamps(None)
    stamped = int((ts.view(-1)[:nblk * 8].view(nblk, 8)[:, 7] > 0).sum())
    P = {k: v.detach().cpu().double() for k, v in enc.state_dict().items()}
    h = torch.nn.functional.gelu(torch.einsum("ec,bchw->behw", P["pwconv1.weight"], torch.from_numpy(x).double())
                                 + P["pwconv1.bias"].view(1, -1, 1, 1))
    m = torch.einsum("ce,behw->bchw", P["pwconv2.weight"], h) + P["pwconv2.bias"].view(1, -1, 1, 1)
    ref = torch.from_numpy(y).double() + P["gamma"].view(1, -1, 1, 1) * m
    tol = 2e-5 * max(1.0, float(m.abs().max()) * gscale)
    err = float((out.double().cpu() - ref).abs().max())
    res[f"{B}x{H}x{W}"] = {"err": err, "tol": tol, "blocks": nblk, "stamped": stamped,
                           "beyond": int((ts.view(-1)[nblk * 8:] != 0).sum())}
print(json.dumps(res))
'''


@pytest.mark.gpu
def test_mlp80_tile_vs_fp64():
    env = dict(os.environ, REPO=REPO, FSMI_MLP_PX="80")
    env.pop("FSMI_LIB", None)
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    for k, v in res.items():
        assert v["err"] <= v["tol"], (k, v)
        assert v["stamped"] == v["blocks"] and v["beyond"] == 0, (k, v)   # exactly the 80-pixel grid ran
