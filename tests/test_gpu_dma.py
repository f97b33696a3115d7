"""Regression test for the pointwise tiles' LDS-DMA ring (csrc/conv_pw.hip dma16).

Round 4 found the DMA's inline asm writing M0 without saving it (the compiler keeps its own value
there) and without the one wait state an M0 write needs before an LDS-DMA: a DMA occasionally used a
stale M0 and filled another ring slot, and about 1 in 40 runs of the split-K pointwise tests saw
wrong partial sums (an eighth of the pixel tiles off).  Here every pointwise tile runs the same
split-K conv many times back to back; all repetitions must be bit-identical and match fp64 torch.
"""
import pytest
import torch
import torch.nn.functional as F

from foundationstereo_amd import synth

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module")
def ops_mod():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from foundationstereo_amd import _lib, ops
    _lib.load()
    return ops


@pytest.mark.parametrize("cfg", [24, 25, 26, 27, 28, 29])
@pytest.mark.parametrize("nsplit", [1, 2, 3])
def test_pw_dma_repeatable(ops_mod, cfg, nsplit):
    B, cin, cout, H, W = 2, 96, 130, 16, 40
    x = torch.from_numpy(synth.normal(881, (B, cin, H, W)))
    w = torch.from_numpy(synth.normal(882, (cout, cin, 1, 1), 0.2))
    pk = ops_mod.PackedConv(w.to(DEV), mode="halo")
    xg = x.to(DEV)
    with torch.no_grad():
        outs = [ops_mod.conv2d([xg], pk, cfg=cfg, nsplit=nsplit) for _ in range(24)]
    torch.cuda.synchronize()
    first = outs[0]
    for o in outs[1:]:
        assert torch.equal(o, first)
    ref = F.conv2d(x.double(), w.double())
    assert float((first.double().cpu() - ref).abs().max() / ref.abs().max()) < 3e-6


# the same matrix in the one-product build (libfsmi_fast.so: round 4's race lived there), in a child
# process since the library is chosen once per process (tests/test_gpu_fast.py); also a single-chunk
# layer (Cin <= 32: the odd tail step right after the prologue) and convc1's 1044-channel shape
CHILD = r'''
import json, os, sys
sys.path.insert(0, os.environ["REPO"])
import torch, torch.nn.functional as F
from foundationstereo_amd import _lib, ops, synth
_lib.load()
dev = torch.device("cuda:0")
worst, bad = 0.0, []
for (B, cin, cout, H, W) in [(2, 96, 130, 16, 40), (1, 32, 64, 8, 40), (1, 1044, 256, 24, 32)]:
    x = torch.from_numpy(synth.normal(881, (B, cin, H, W)))
    w = torch.from_numpy(synth.normal(882, (cout, cin, 1, 1), 0.2))
    pk = ops.PackedConv(w.to(dev), mode="halo")
    xg = x.to(dev)
    ref = F.conv2d(x.double(), w.double())
    for cfg in (24, 25, 26, 27, 28, 29):
        for nsplit in (1, 2, 3):
            with torch.no_grad():
                outs = [ops.conv2d([xg], pk, cfg=cfg, nsplit=nsplit) for _ in range(24)]
            torch.cuda.synchronize()
            same = all(torch.equal(o, outs[0]) for o in outs[1:])
            err = float((outs[0].double().cpu() - ref).abs().max() / ref.abs().max())
            worst = max(worst, err)
            if not same or not err < float(os.environ["TOL"]):
                bad.append((cin, cfg, nsplit, same, err))
print(json.dumps({"lib": os.path.basename(_lib.library_path()), "worst": worst, "bad": bad}))
'''


@pytest.mark.parametrize("precision,tol", [("fast", 5e-3), ("parity", 1e-5)])
def test_pw_dma_repeatable_child(precision, tol):
    import json
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    env = dict(os.environ, REPO=repo, FSMI_PRECISION=precision, TOL=str(tol))
    env.pop("FSMI_LIB", None)
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["lib"] == ("libfsmi_fast.so" if precision == "fast" else "libfsmi.so"), res
    assert not res["bad"], res
    print(f"{precision}: worst relative error {res['worst']:.2e}")
