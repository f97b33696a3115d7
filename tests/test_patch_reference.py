"""The Python drop-in seam on the unmodified reference, CPU only.

``foundationstereo_amd.patch_reference(core.foundation_stereo)`` must make the reference's own
``FoundationStereo`` build this package's modules (update block, 3D filtering blocks,
hourglass + disparity transformer, context net, geometry encoding) and accept a state dict
strictly.  Runs ``tools/check_patch_reference.py`` in a subprocess (the reference import stubs
absent third-party packages into ``sys.modules``); skipped where the reference is absent (the
GPU box)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.environ.get("FSMI_REFERENCE", "/root/reference")


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "core")), reason="reference not present")
def test_patch_reference_rebinds_and_loads():
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "check_patch_reference.py")], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["state_equal"] and res["n_keys"] > 500
    for name in ("build_gwc_volume", "build_concat_volume", "disparity_regression", "BasicSelectiveMultiUpdateBlock",
                 "BasicConv", "Conv3dNormActReduced", "ResnetBasicBlock3D", "FeatureAtt",
                 "CostVolumeDisparityAttention", "ContextNetDino", "hourglass", "Combined_Geo_Encoding_Volume",
                 "InputPadder", "bilinear_sampler"):
        assert name in res["replaced"], name
    for what, mod in res["modules"].items():
        assert mod.startswith("foundationstereo_amd."), (what, mod)
