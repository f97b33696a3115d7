"""GPU parity of the disparity-transformer kernels (csrc/transformer.hip)
against the same ops in fp64 PyTorch on the CPU:

* conv_patch (depthwise Conv3d k4 s4 + eval BatchNorm3d, core/foundation_stereo.py:85-88);
* CostVolumeDisparityAttention (core/submodule.py:506-528) -- PE, 4 post-norm encoder layers with
  4-head softmax attention and an exact-GELU FFN -- run through the module's own torch path;
* the x4 trilinear (align_corners=False) upsample-and-add (core/foundation_stereo.py:119-120).

fp32 kernels vs fp64 references: abs 2e-5 (patch / upsample: summation order only), abs 1e-4 for
the 4-layer transformer (LayerNorm renormalises, errors do not grow layer to layer).
"""
import numpy as np
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


@pytest.fixture(scope="module")
def ops_mod():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from foundationstereo_amd import _lib, ops
    _lib.load()
    return ops


def _close(a, b, atol):
    np.testing.assert_allclose(a.detach().double().cpu().numpy(), b.detach().double().cpu().numpy(), atol=atol,
                               rtol=0)


def _seeded(mod, seed):
    gen = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for p in mod.parameters():
            p.copy_(torch.randn(p.shape, generator=gen) * (0.3 if p.dim() > 1 else 0.1))
        for m in mod.modules():
            if isinstance(m, nn.LayerNorm):
                m.weight.add_(1.0)
    return mod


@pytest.mark.parametrize("shape", [(1, 28, 48, 16, 24), (2, 28, 16, 8, 12), (1, 5, 8, 4, 4)])
def test_patch_embed_vs_torch(ops_mod, shape):
    B, C, D, H, W = shape
    gen = torch.Generator().manual_seed(11)
    x = torch.randn(shape, generator=gen)
    conv = nn.Conv3d(C, C, 4, stride=4, groups=C)
    bn = nn.BatchNorm3d(C).eval()
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=gen) * 0.2)
        conv.bias.copy_(torch.randn(C, generator=gen) * 0.1)
        bn.weight.copy_(torch.rand(C, generator=gen) + 0.5)
        bn.bias.copy_(torch.randn(C, generator=gen) * 0.1)
        bn.running_mean.copy_(torch.randn(C, generator=gen) * 0.1)
        bn.running_var.copy_(torch.rand(C, generator=gen) + 0.5)
        ref = bn.double()(conv.double()(x.double()))
        inv = (bn.running_var + bn.eps).rsqrt() * bn.weight
        shift = (conv.bias - bn.running_mean) * inv + bn.bias
        out = ops_mod.dt_patch_embed(x.float().to(DEV), conv.weight.float().to(DEV), inv.float().to(DEV),
                                     shift.float().to(DEV))
    _close(out, ref, 2e-5)


@pytest.mark.parametrize("L,H,W,B", [(12, 3, 5, 2), (20, 2, 3, 1), (5, 4, 7, 1), (64, 2, 2, 1), (1, 3, 3, 1)])
def test_disparity_transformer_vs_torch(ops_mod, L, H, W, B):
    from foundationstereo_amd.submodule import CostVolumeDisparityAttention
    mod = _seeded(CostVolumeDisparityAttention(d_model=28, nhead=4, dim_feedforward=28, num_transformer=4,
                                               max_len=max(L, 12)), 5 + L).eval()
    gen = torch.Generator().manual_seed(7)
    cv = torch.randn(B, 28, L, H, W, generator=gen)
    with torch.no_grad():
        ref = mod.double()(cv.double())                     # CPU: the module's torch path
        mod.float().to(DEV)
        assert mod._fast(cv.to(DEV))
        out = mod(cv.to(DEV))
    _close(out, ref, 1e-4)


def test_disparity_transformer_rejects_other_widths(ops_mod):
    from foundationstereo_amd._lib import FsmiError
    x = torch.zeros(1, 32, 4, 2, 2, device=DEV)
    with pytest.raises(FsmiError):
        ops_mod.disparity_transformer(x, torch.zeros(10, device=DEV), torch.zeros(4, 32, device=DEV), 4, 32, 1)


@pytest.mark.parametrize("shape", [(1, 28, 12, 30, 40), (2, 3, 2, 3, 5), (1, 2, 1, 1, 1)])
def test_upsample4_add_vs_torch(ops_mod, shape):
    gen = torch.Generator().manual_seed(3)
    t_ = torch.randn(shape, generator=gen)
    B, C, D, H, W = shape
    vol = torch.randn(B, C, 4 * D, 4 * H, 4 * W, generator=gen)
    ref = vol.double() + F.interpolate(t_.double(), scale_factor=4, mode="trilinear", align_corners=False)
    out = vol.to(DEV)
    ops_mod.upsample4_add_(out, t_.to(DEV))
    _close(out, ref, 2e-5)


def test_hourglass_dt_fast_matches_torch_path(ops_mod, monkeypatch):
    """The hourglass tail (conv_patch -> transformer -> x4 add) with the HIP kernels vs the same
    module with them disabled, at cfg1-like sizes."""
    from foundationstereo_amd import submodule
    from foundationstereo_amd.foundation_stereo import hourglass
    hg = hourglass({"max_disp": 64}, 28, [128, 192, 320, 304])
    hg = _seeded(hg, 21).eval()
    with torch.no_grad():
        for m in hg.modules():
            if isinstance(m, nn.BatchNorm3d):
                m.running_var.fill_(1.0)
    hg.to(DEV)
    gen = torch.Generator().manual_seed(4)
    x = torch.randn(1, 28, 16, 32, 32, generator=gen).to(DEV)
    feats = [None, torch.randn(1, 192, 16, 16, generator=gen).to(DEV), torch.randn(1, 320, 8, 8, generator=gen).to(DEV),
             torch.randn(1, 304, 4, 4, generator=gen).to(DEV)]
    with torch.no_grad():
        fast = hg(x, feats)
        monkeypatch.setattr(submodule, "DT_FAST", False)
        slow = hg(x, feats)
    _close(fast, slow, 1e-3 * max(1.0, float(slow.abs().max())))
