"""Checkpoint / cfg loading (scripts/run_demo.py:111-125) on the CPU: a checkpoint written in the
reference's layout ({'model': state_dict, 'global_step', 'epoch'} + cfg.yaml beside it) loads
strictly into a fresh model; a missing key or a wrong vit_size fails loudly."""
import os

import pytest
import torch
import yaml

from foundationstereo_amd import synth
from foundationstereo_amd.checkpoint import load_cfg, load_model


def _write(tmp_path, vit="vits", cfg_extra=None, drop=None, extra=None):
    from foundationstereo_amd.foundation_stereo import FoundationStereo
    args = synth.make_args(max_disp=64, corr_levels=2, vit_size=vit)
    m = FoundationStereo(args)
    synth.init_module_(m, seed=7)
    sd = m.state_dict()
    if drop:
        sd = {k: v for k, v in sd.items() if k != drop}
    if extra:
        sd = dict(sd, **extra)
    path = os.path.join(tmp_path, "model_best_bp2.pth")
    torch.save({"model": sd, "global_step": 123, "epoch": 4}, path)
    cfg = dict(args)
    cfg.update(cfg_extra or {})
    with open(os.path.join(tmp_path, "cfg.yaml"), "w") as f:
        yaml.safe_dump(cfg, f)
    return path, m


def test_load_model_roundtrip(tmp_path):
    path, ref = _write(tmp_path)
    model, meta = load_model(path, overrides={"valid_iters": 8})
    assert meta == {"global_step": 123, "epoch": 4, "skipped_backbone_keys": []}
    assert not model.training and model.args.valid_iters == 8 and model.args.get("vit_size") == "vits"
    a, b = model.state_dict(), ref.state_dict()
    assert list(a) == list(b)
    for k in a:
        assert torch.equal(a[k], b[k]), k


def test_cfg_defaults_vit_size_to_vitl(tmp_path):
    path, _ = _write(tmp_path)
    cfg = {k: v for k, v in synth.make_args(max_disp=64, corr_levels=2).items() if k != "vit_size"}
    with open(os.path.join(tmp_path, "cfg.yaml"), "w") as f:
        yaml.safe_dump(cfg, f)
    assert load_cfg(path)["vit_size"] == "vitl"
    with pytest.raises(RuntimeError):          # a ViT-S checkpoint does not fit the ViT-L tree
        load_model(path)


def test_missing_key_is_an_error(tmp_path):
    path, ref = _write(tmp_path, drop="classifier.2.weight")
    with pytest.raises(RuntimeError, match="classifier"):
        load_model(path)


def test_backbone_keys_are_set_aside(tmp_path):
    """A real checkpoint holds the backbone's ``feature.*`` weights; with the parameter-free
    synthetic backbone they are reported and everything else still loads strictly."""
    extra = {"feature.stem.0.weight": torch.zeros(48, 3, 4, 4),
             "feature.dino.blocks.0.norm1.weight": torch.ones(384)}
    path, ref = _write(tmp_path, extra=extra)
    model, meta = load_model(path)
    assert sorted(meta["skipped_backbone_keys"]) == sorted(extra)
    a, b = model.state_dict(), ref.state_dict()
    assert list(a) == list(b) and all(torch.equal(a[k], b[k]) for k in a)


def test_unexpected_non_backbone_key_is_an_error(tmp_path):
    path, _ = _write(tmp_path, extra={"update_block.bogus.weight": torch.zeros(3)})
    with pytest.raises(RuntimeError, match="bogus"):
        load_model(path)


def test_backbone_keys_load_into_real_feature(tmp_path):
    """With the real backbone (backbone=True) the checkpoint's feature.* weights load strictly."""
    from foundationstereo_amd.foundation_stereo import FoundationStereo
    args = synth.make_args(max_disp=64, corr_levels=2, vit_size="vits")
    args["backbone"] = "real"
    m = FoundationStereo(args)
    synth.init_module_(m, seed=7)
    path = os.path.join(tmp_path, "model_best_bp2.pth")
    torch.save({"model": m.state_dict(), "global_step": 1, "epoch": 0}, path)
    cfg = {k: v for k, v in args.items() if k != "backbone"}
    with open(os.path.join(tmp_path, "cfg.yaml"), "w") as f:
        yaml.safe_dump(cfg, f)
    model, meta = load_model(path, backbone=True)
    assert meta["skipped_backbone_keys"] == []
    a, b = model.state_dict(), m.state_dict()
    assert list(a) == list(b) and any(k.startswith("feature.dino.") for k in a)
    assert all(torch.equal(a[k], b[k]) for k in a)
