"""Checkpoint + config loading of ``scripts/run_demo.py:111-125``.

The reference reads ``cfg.yaml`` next to the checkpoint with OmegaConf, defaults
``vit_size`` to ``vitl``, overlays the command-line args, builds
``FoundationStereo(args)`` and loads ``torch.load(ckpt)['model']``.  OmegaConf is
absent from this image: ``cfg.yaml`` is plain YAML, read with ``yaml.safe_load``
into a ``StereoArgs`` (attribute, item and ``.get`` access, as OmegaConf gives).
The checkpoint is read with ``weights_only=True``: tensors and plain containers
only, nothing in the file is executed.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch
import yaml

from .synth import StereoArgs


def load_cfg(ckpt_path: str, overrides: Optional[dict] = None) -> StereoArgs:
    """``cfg.yaml`` beside ``ckpt_path`` (scripts/run_demo.py:112-117)."""
    cfg_path = os.path.join(os.path.dirname(os.path.abspath(ckpt_path)), "cfg.yaml")
    with open(cfg_path) as f:
        cfg = yaml.safe_load(f) or {}
    if not isinstance(cfg, dict):
        raise ValueError(f"{cfg_path}: expected a mapping, got {type(cfg).__name__}")
    cfg.setdefault("vit_size", "vitl")
    cfg.update(overrides or {})
    return StereoArgs(cfg)


def load_model(ckpt_path: str, overrides: Optional[dict] = None, device=None,
               feature=None, backbone: bool = False) -> Tuple[torch.nn.Module, dict]:
    """FoundationStereo with the checkpoint's ``model`` state loaded strictly, in eval mode
    (scripts/run_demo.py:121-129).  Returns (model, meta): meta holds the checkpoint's
    ``global_step`` / ``epoch`` and ``skipped_backbone_keys``.

    A real checkpoint carries the backbone's ``feature.*`` weights (EdgeNeXt + DepthAnythingV2).  When ``feature`` is None (the parameter-free synthetic
    stand-in) or has no parameters of its own, those keys cannot be loaded anywhere: they are
    set aside and listed in ``meta["skipped_backbone_keys"]``, and every other key still loads
    strictly.  With a backbone that has parameters (``backbone=True``: the real ``Feature``,
    core/extractor.py:323-369), ``feature.*`` must match it exactly."""
    from .foundation_stereo import FoundationStereo
    args = load_cfg(ckpt_path, overrides)
    if backbone and feature is None:
        from .backbone import Feature
        feature = Feature(args)
    model = FoundationStereo(args, feature=feature)
    ckpt = torch.load(ckpt_path, map_location="cpu", weights_only=True)
    if not isinstance(ckpt, dict) or "model" not in ckpt:
        raise KeyError(f"{ckpt_path}: no 'model' state in the checkpoint")
    state = ckpt["model"]
    skipped = []
    if not any(True for _ in model.feature.state_dict()):
        skipped = [k for k in state if k.startswith("feature.")]
        state = {k: v for k, v in state.items() if not k.startswith("feature.")}
    model.load_state_dict(state)
    model.eval()
    if device is not None:
        model.to(device)
    meta = {k: ckpt.get(k) for k in ("global_step", "epoch")}
    meta["skipped_backbone_keys"] = skipped
    return model, meta
