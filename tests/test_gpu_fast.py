"""The opt-in reference-precision build (FSMI_PRECISION=fast, _lib/libfsmi_fast.so: one fp16 MFMA
product per conv MAC, csrc/conv_halo.h FSMI_NPROD=1) on the GPU.

The library is chosen once per process, so the fast forward runs in a child process.  It is NOT held
to the 1e-3 px parity bar (that is the 3-product default's); the test pins that the child really ran
the fast build (its disparity differs from the parity build's) and bounds its error against the CPU
oracle at the size of fp16-autocast drift."""
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
import oracle
from foundationstereo_amd import _lib, synth
from foundationstereo_amd.foundation_stereo import FoundationStereo
lib = _lib.load()
H, W, md, iters, L = 64, 96, 32, 4, 2
args = synth.make_args(max_disp=md, corr_levels=L, vit_size="vits")
model = FoundationStereo(args).eval()
synth.init_module_(model, seed=1234)
fl, fr, vf = synth.backbone_features(1, H, W, "vits", shift_px=2)
left, right = synth.stereo_images(1, H, W)
dev = torch.device("cuda:0")
model = model.to(dev)
model.feature.set_features([torch.from_numpy(a).to(dev) for a in fl], [torch.from_numpy(a).to(dev) for a in fr],
                           torch.from_numpy(vf).to(dev))
with torch.no_grad():
    out = model(torch.from_numpy(left).to(dev), torch.from_numpy(right).to(dev), iters=iters, test_mode=True)
out = out.float().cpu()
P = {k: v.detach().float().cpu() if v.is_floating_point() else v.cpu() for k, v in model.state_dict().items()}
with torch.no_grad():
    ref = oracle.oracle_forward(P, args, torch.from_numpy(left), torch.from_numpy(right),
                                [torch.from_numpy(a) for a in fl], [torch.from_numpy(a) for a in fr],
                                torch.from_numpy(vf), iters=iters)
np.save(os.environ["OUT"], out.numpy())
print(json.dumps({"lib": os.path.basename(_lib.library_path()), "dd": float((out - ref).abs().max()),
                  "mean": float(out.mean())}))
'''


def _run(precision, tmp_path):
    env = dict(os.environ, REPO=REPO, FSMI_PRECISION=precision, OUT=str(tmp_path / f"{precision}.npy"))
    env.pop("FSMI_LIB", None)
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.gpu
def test_fast_precision_build(tmp_path):
    import numpy as np
    from foundationstereo_amd import build
    if not os.path.exists(build.LIB_FAST):
        pytest.fail("libfsmi_fast.so not built (__graft_entry__.build())")
    fast = _run("fast", tmp_path)
    par = _run("parity", tmp_path)
    assert fast["lib"] == "libfsmi_fast.so" and par["lib"] == "libfsmi.so"
    assert par["dd"] < 1e-3, par                                  # the default keeps parity
    a, b = np.load(tmp_path / "fast.npy"), np.load(tmp_path / "parity.npy")
    assert np.isfinite(a).all()
    assert float(np.abs(a - b).max()) > 0.0                      # a different (1-product) conv path ran
    assert fast["dd"] < 0.25, fast                                # fp16-autocast-sized drift, not garbage
    print(f"fast |dd| vs oracle {fast['dd']:.2e} px, parity {par['dd']:.2e} px")
