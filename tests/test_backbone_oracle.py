"""CPU: the backbone oracle (oracle/backbone_oracle.py) vs goldens made by the REFERENCE
(tools/make_goldens.py ``backbone``: DepthAnythingFeature vits / vitl and Feature with the module-form
timm restatement), and the product module trees vs the reference's state_dict keys, shapes and order."""
import json
import os

import numpy as np
import pytest
import torch

from foundationstereo_amd import backbone as bb, synth
from oracle import backbone_oracle as bo

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _gold(name):
    return np.load(os.path.join(GOLD, name + ".npz"))


def _params(module, seed=4321):
    sd = module.state_dict()
    vals = synth.init_state([(k, tuple(v.shape)) for k, v in sd.items()], seed=seed)
    return {k: torch.from_numpy(np.asarray(v)).float() for k, v in vals.items()}


@pytest.mark.parametrize("name,ctor", [
    ("dav2_vits", lambda: bb.DepthAnythingFeature("vits")),
    ("dav2_vitl", lambda: bb.DepthAnythingFeature("vitl")),
    ("feature_vits", lambda: bb.Feature(synth.make_args(vit_size="vits"))),
])
def test_state_dict_matches_reference(name, ctor):
    with open(os.path.join(GOLD, f"state_dict_{name}.json")) as f:
        ref = json.load(f)
    mine = [[k, list(v.shape)] for k, v in ctor().state_dict().items()]
    assert [k for k, _ in mine] == [k for k, _ in ref]
    assert mine == ref


def _close(a, b, rtol=2e-5, atol=2e-5):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    scale = max(1.0, float(np.abs(b).max()))
    err = float(np.abs(a - b).max())
    assert err <= atol * scale + rtol * float(np.abs(b).max()), f"max |diff| {err:.3g} (scale {scale:.3g})"
    return err


@pytest.mark.parametrize("name,enc", [("dav2_vits", "vits"), ("dav2_vitl", "vitl")])
def test_depth_anything_oracle_vs_reference(name, enc):
    g = _gold(name)
    P = _params(bb.DepthAnythingFeature(enc))
    shape = {"dav2_vits": (2, 3, 56, 70), "dav2_vitl": (1, 3, 28, 42)}[name]
    x = torch.from_numpy(synth.normal(synth.name_seed(name + "_x"), shape))
    with torch.no_grad():
        out = bo.depth_anything_feature(P, "", x, enc)
    for k in ("out", "path_1", "path_2", "path_3", "path_4", "disp"):
        _close(out[k].numpy(), g[k])
    for i, (tok, cls) in enumerate(out["features"]):
        _close(tok.numpy(), g[f"feat{i}"])
        _close(cls.numpy(), g[f"cls{i}"])


def test_feature_oracle_vs_reference():
    g = _gold("feature_vits")
    P = _params(bb.Feature(synth.make_args(vit_size="vits")))
    x = torch.from_numpy(synth.normal(synth.name_seed("feature_vits_x"), (2, 3, 64, 96)))
    with torch.no_grad():
        feats, vit_feat = bo.feature_forward(P, "", x, "vits")
    for i, f in enumerate(feats):
        _close(f.numpy(), g[f"x{4 << i}"])
    _close(vit_feat.numpy(), g["vit_feat"])


def test_resize_keep_aspect_matches_utils():
    # Utils.py:89-105 at the benchmark sizes (lcm(14, 16) = 112, cap 1344)
    assert bb.get_resize_keep_aspect_ratio(480, 640, 112, 1344, 1344) == (560, 672)
    assert bo.resize_keep_aspect(1024, 1536, 112, 1344, 1344) == bb.get_resize_keep_aspect_ratio(1024, 1536, 112, 1344,
                                                                                                 1344)
    assert bb.get_resize_keep_aspect_ratio(384, 1248, 112, 1344, 1344) == (448, 1344)


@pytest.mark.parametrize("vit", ["vits", "vitl"])
def test_full_model_state_dict_with_backbone(vit):
    """FoundationStereo with the real backbone: every key of the reference checkpoint layout (feature.*
    included), same shapes, same order (core/foundation_stereo.py:127-180)."""
    from foundationstereo_amd.foundation_stereo import FoundationStereo
    with open(os.path.join(GOLD, f"state_dict_full_{vit}.json")) as f:
        ref = json.load(f)
    args = synth.make_args(max_disp=192, corr_levels=4, vit_size=vit)
    args["backbone"] = "real"
    mine = [[k, list(v.shape)] for k, v in FoundationStereo(args).state_dict().items()]
    assert mine == ref
