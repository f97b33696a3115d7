"""Import the reference FoundationStereo modules read-only, in THIS container only.

Used by ``tools/make_goldens.py`` to produce golden vectors; never imported by
the product, the GPU tests, ``smoke()`` or ``bench.py`` (the reference does not
exist on the GPU box).

Absent third-party modules that carry no hot-path arithmetic are stubbed
(SURVEY.md §8c): open3d, trimesh, transformations, imageio, cv2,
torchvision (``transforms.Normalize`` only) and flash_attn (``flash_attn_func``
restated as non-causal SDPA with the default 1/sqrt(head_dim) scale, the same
math as the reference's call at ``core/submodule.py:224``).  For the stereo goldens the backbone
``Feature`` (remote timm / torch.hub weights) is replaced by a synthetic source; for the backbone
goldens ``torch.hub.load`` builds DINOv2 from the vendored ``dinov2/`` (pretrained=False) and
``timm.create_model('edgenext_small')`` returns tools/edgenext_timm.py's restatement (no weights).
"""
from __future__ import annotations

import os
import sys
import types

REF_ROOT = os.environ.get("FSMI_REFERENCE", "/root/reference")


def _stub(name, **attrs):
    m = types.ModuleType(name)
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


def install_stubs():
    import torch
    import torch.nn.functional as F

    for n in ("open3d", "trimesh", "transformations", "imageio"):
        if n not in sys.modules:
            _stub(n)
    if "timm" not in sys.modules:
        # core/extractor.py:327 timm.create_model('edgenext_small', pretrained=True): answered by the
        # module-form restatement of timm's published edgenext_small (tools/edgenext_timm.py; no weights)
        def create_model(*a, **k):
            sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
            import edgenext_timm
            return edgenext_timm.create_model(*a, **k)
        _stub("timm", create_model=create_model)
    if "cv2" not in sys.modules:
        _stub("cv2", COLORMAP_TURBO=20, COLORMAP_JET=2)

    class Normalize:
        def __init__(self, mean, std, inplace=False):
            self.mean = torch.tensor(mean).view(-1, 1, 1)
            self.std = torch.tensor(std).view(-1, 1, 1)

        def __call__(self, x):
            return (x - self.mean.to(x)) / self.std.to(x)

    if "torchvision" not in sys.modules:
        tv = _stub("torchvision")
        tr = _stub("torchvision.transforms", Normalize=Normalize)
        tv.transforms = tr

    def flash_attn_func(q, k, v, window_size=(-1, -1), **_):
        o = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2))
        return o.transpose(1, 2)

    if "flash_attn" not in sys.modules:
        _stub("flash_attn", flash_attn_func=flash_attn_func,
              flash_attn_qkvpacked_func=lambda *a, **k: (_ for _ in ()).throw(NotImplementedError()))


def install_hub_stub():
    """depth_anything/dpt.py:159 fetches DINOv2 with torch.hub.load('facebookresearch/dinov2', ...) (remote);
    answer it from the vendored copy in the reference, the way dinov2/hub/backbones.py:18-61 builds the
    model (pretrained=False: no weight download)."""
    import torch
    if os.path.join(REF_ROOT, "dinov2") not in sys.path:
        sys.path.insert(0, os.path.join(REF_ROOT, "dinov2"))
    from dinov2.hub import backbones

    def hub_load(repo, model, *a, pretrained=True, **k):
        assert repo == "facebookresearch/dinov2", repo
        return getattr(backbones, model)(pretrained=False, **k)

    torch.hub.load = hub_load


def import_reference():
    """Return the reference modules ``(foundation_stereo, submodule, geometry, update, utils)``."""
    sys.dont_write_bytecode = True
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    install_stubs()
    if REF_ROOT not in sys.path:
        sys.path.insert(0, REF_ROOT)
    import importlib
    fs = importlib.import_module("core.foundation_stereo")
    sm = importlib.import_module("core.submodule")
    geo = importlib.import_module("core.geometry")
    up = importlib.import_module("core.update")
    ut = importlib.import_module("core.utils.utils")
    return fs, sm, geo, up, ut


def import_reference_extractor():
    """The reference ``core.extractor`` (Feature, DepthAnythingFeature) with the hub / timm stand-ins."""
    import_reference()
    install_hub_stub()
    import importlib
    return importlib.import_module("core.extractor")


def make_synthetic_feature_class(feature_dims_fn):
    """A drop-in for ``core.extractor.Feature`` returning preset tensors."""
    import torch.nn as nn
    import torch

    class SyntheticFeature(nn.Module):
        def __init__(self, args):
            super().__init__()
            self.d_out, self.vit_dim = feature_dims_fn(args.vit_size)
            self.preset = None
            self.by_size = None      # (vit_size, shift_px): synthesise for the input size instead

        def forward(self, x):
            if self.by_size is not None:
                from foundationstereo_amd import synth
                B2, _, H, W = x.shape
                fl, fr, vit = synth.backbone_features(B2 // 2, H, W, self.by_size[0], shift_px=self.by_size[1])
                fl, fr, vit = [torch.from_numpy(a) for a in fl], [torch.from_numpy(a) for a in fr], \
                    torch.from_numpy(vit)
            else:
                fl, fr, vit = self.preset
            out = [torch.cat([a, b], 0) for a, b in zip(fl, fr)]
            return out, torch.cat([vit, vit], 0)

    return SyntheticFeature
