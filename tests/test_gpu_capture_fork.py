"""The pipelined refinement loop (update.BasicSelectiveMultiUpdateBlock.run_pipelined) captured into a
hipGraph with its optional stream forks, each in a child process (the knobs are read at import; a crash
under capture must fail this test, not the runner):

  * default: gru04's small branch on the branch stream (FSMI_PIPE_BRANCH=1);
  * everything in order on its stream (FSMI_PIPE_BRANCH=0);
  * FSMI_MOTION_ON_MAIN=1: the motion path on the main stream.

Every configuration runs the same kernels on the same inputs, so the eager forward and the replayed
graph must be bit-identical across all of them.  faulthandler prints the Python stack of a segfault.
Forking gru08's small branch from the pipeline stream (round 4's segfault) breaks the capture_fork rule
(update.py): tools/capture_fork_probe.py reproduces that crash with plain torch ops; update.stream_wait
now raises CaptureForkError before such a capture can end (tests/test_capture_fork_guard.py, and the
last test here forces it under a real capture); the middle test runs the probe's passing patterns."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import faulthandler, json, os, sys
faulthandler.enable()
sys.path.insert(0, os.environ["REPO"])
import numpy as np, torch
from foundationstereo_amd import _lib, synth
from foundationstereo_amd.foundation_stereo import FoundationStereo
_lib.load()
H, W, md, iters = 64, 96, 32, 4
args = synth.make_args(max_disp=md, corr_levels=2, vit_size="vits")
model = FoundationStereo(args).eval()
synth.init_module_(model, seed=1234)
fl, fr, vf = synth.backbone_features(1, H, W, "vits", shift_px=2)
left, right = synth.stereo_images(1, H, W)
dev = torch.device("cuda:0")
model = model.to(dev)
model.feature.set_features([torch.from_numpy(a).to(dev) for a in fl], [torch.from_numpy(a).to(dev) for a in fr],
                           torch.from_numpy(vf).to(dev))
L, R = torch.from_numpy(left).to(dev), torch.from_numpy(right).to(dev)
with torch.no_grad():
    eager = model(L, R, iters=iters, test_mode=True).float().cpu().numpy()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = model(L, R, iters=iters, test_mode=True)
g.replay()
g.replay()
torch.cuda.synchronize()
rep = out.float().cpu().numpy()
np.save(os.environ["OUT"] + "_eager.npy", eager)
np.save(os.environ["OUT"] + "_graph.npy", rep)
print(json.dumps({"finite": bool(np.isfinite(rep).all()), "mean": float(rep.mean())}))
'''

CONFIGS = {
    "default": {},
    "in_order": {"FSMI_PIPE_BRANCH": "0"},
    "motion_on_main": {"FSMI_MOTION_ON_MAIN": "1"},
}


def _run(name, tmp_path):
    env = dict(os.environ, REPO=REPO, OUT=str(tmp_path / name), **CONFIGS[name])
    for k in ("FSMI_PIPE_BRANCH", "FSMI_MOTION_ON_MAIN"):
        if k not in CONFIGS[name]:
            env.pop(k, None)
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, f"{name}: exit {r.returncode}\n{r.stderr[-3000:]}"
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.gpu
def test_pipelined_capture_forks(tmp_path):
    res = {name: _run(name, tmp_path) for name in CONFIGS}
    ref = np.load(tmp_path / "in_order_eager.npy")
    for name in CONFIGS:
        assert res[name]["finite"], name
        for kind in ("eager", "graph"):
            got = np.load(tmp_path / f"{name}_{kind}.npy")
            assert np.array_equal(got, ref), f"{name} {kind}: max |d| {float(np.abs(got - ref).max())}"


@pytest.mark.gpu
def test_capture_fork_rule_patterns():
    """The patterns the capture_fork rule allows capture and replay correctly (plain torch ops)."""
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import capture_fork_probe as probe
    for v in ("main_only", "via_main", "via_main_nojoin"):
        r = subprocess.run([sys.executable, "-c", probe.CHILD, v], capture_output=True, text=True, timeout=180)
        assert r.returncode == 0, f"{v}: exit {r.returncode}\n{r.stderr[-2000:]}"
        assert json.loads(r.stdout.strip().splitlines()[-1])["ok"], v


@pytest.mark.gpu
def test_guard_raises_under_real_capture():
    """Forking gru08's small branch from the pipeline stream -- round 4's segfault -- raises
    CaptureForkError inside the capture instead of reaching hipStreamEndCapture (child process)."""
    code = CHILD.replace("with torch.cuda.graph(g):\n        out = model(L, R, iters=iters, test_mode=True)",
                         "from foundationstereo_amd import update as U\n"
                         "    real = U.SelectiveConvGRU.forward\n"
                         "    def fwd(self, *a, **k):\n"
                         "        U._BRANCH[0] = 1\n"
                         "        return real(self, *a, **k)\n"
                         "    U.SelectiveConvGRU.forward = fwd\n"
                         "    try:\n"
                         "        with torch.cuda.graph(g):\n"
                         "            out = model(L, R, iters=iters, test_mode=True)\n"
                         "    except Exception as e:\n"
                         "        c, found = e, False\n"
                         "        while c is not None:\n"
                         "            found, c = found or isinstance(c, U.CaptureForkError), c.__context__\n"
                         "        print(json.dumps({'raised': found})); sys.exit(0)\n"
                         "    print(json.dumps({'raised': None})); sys.exit(0)")
    env = dict(os.environ, REPO=REPO, OUT="/tmp/fsmi_guard")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, f"exit {r.returncode}\n{r.stderr[-3000:]}"
    assert json.loads(r.stdout.strip().splitlines()[-1])["raised"], r.stdout[-500:]
