"""Functional fp32 CPU restatement of the stereo backbone ``Feature`` (core/extractor.py:286-369).

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).  Parameters are looked up by their reference
``state_dict`` names in a flat dict ``P`` (as ``stereo_oracle``).

* DINOv2 ViT (dinov2/dinov2/models/vision_transformer.py:180-323, layers/block.py:89-114,
  layers/attention.py:69-79, layers/patch_embed.py:68-81) and the DPT head
  (depth_anything/dpt.py:105-146, depth_anything/blocks.py:37-153): pinned by goldens generated from
  the reference itself (tools/make_goldens.py ``backbone``).
* EdgeNeXt-S: timm's ``edgenext_small`` (core/extractor.py:327) restated from its published
  architecture (timm is not installed here): PARITY UNPINNED against timm -- the goldens pin it only
  against a second, module-form restatement (tools/edgenext_timm.py) run inside the reference's
  ``Feature``.
* ``Feature.forward`` (core/extractor.py:348-369): pinned by the same goldens (reference code for the
  resize, the DepthAnything features and the Conv2x_IN / conv4 fusion).
"""
from __future__ import annotations

import math
from typing import Dict, List, Sequence

import numpy as np
import torch
import torch.nn.functional as F

from .stereo_oracle import _conv, _deconv, _inorm, _lrelu

Tensor = torch.Tensor
Params = Dict[str, Tensor]

__all__ = ["vit_intermediate", "dpt_head", "depth_anything_feature", "edgenext_trunk", "feature_forward",
           "resize_keep_aspect"]

_VIT = {"vits": (384, 12, 6), "vitb": (768, 12, 12), "vitl": (1024, 24, 16)}
_IDX = {"vits": [2, 5, 8, 11], "vitb": [2, 5, 8, 11], "vitl": [4, 11, 17, 23]}
_CFG = {"vits": (64, [48, 96, 192, 384]), "vitb": (128, [96, 192, 384, 768]), "vitl": (256, [256, 512, 1024, 1024])}


def _ln(P, name, x, eps=1e-6):
    return F.layer_norm(x, (x.shape[-1],), P[name + ".weight"], P[name + ".bias"], eps)


def _lin(P, name, x):
    return F.linear(x, P[name + ".weight"], P.get(name + ".bias"))


# ----------------------------------------------------------------------------
# DINOv2 ViT
# ----------------------------------------------------------------------------

def _pos_embed(P, p, ph, pw, offset=0.1):
    """interpolate_pos_encoding, vision_transformer.py:180-212 (bicubic with scale factors)."""
    pos = P[p + "pos_embed"].float()
    N0 = pos.shape[1] - 1
    M = int(math.sqrt(N0))
    if N0 == ph * pw and ph == pw:
        return pos
    D = pos.shape[-1]
    g = F.interpolate(pos[:, 1:].reshape(1, M, M, D).permute(0, 3, 1, 2), mode="bicubic", antialias=False,
                      scale_factor=(float(ph + offset) / M, float(pw + offset) / M))
    return torch.cat([pos[:, :1], g.permute(0, 2, 3, 1).reshape(1, -1, D)], 1)


def vit_intermediate(P: Params, p: str, x: Tensor, idx: Sequence[int], heads: int):
    """get_intermediate_layers(x, idx, return_class_token=True) (vision_transformer.py:273-323): a list of
    (normalised patch tokens (B, N, D), normalised class token (B, D))."""
    w = P[p + "patch_embed.proj.weight"]
    ps = w.shape[-1]
    B, _, H, W = x.shape
    ph, pw = H // ps, W // ps
    t = F.conv2d(x, w, P[p + "patch_embed.proj.bias"], stride=ps).flatten(2).transpose(1, 2)   # (B, N, D)
    t = torch.cat([P[p + "cls_token"].expand(B, -1, -1), t], 1) + _pos_embed(P, p, ph, pw)
    D = t.shape[-1]
    hd = D // heads
    out = []
    i = 0
    while f"{p}blocks.{i}.norm1.weight" in P:
        b = f"{p}blocks.{i}."
        h = _ln(P, b + "norm1", t)
        qkv = _lin(P, b + "attn.qkv", h).reshape(B, -1, 3, heads, hd).permute(2, 0, 3, 1, 4)
        a = F.scaled_dot_product_attention(qkv[0], qkv[1], qkv[2])           # attention.py:74-77
        a = a.transpose(1, 2).reshape(B, -1, D)
        t = t + P[b + "ls1.gamma"] * _lin(P, b + "attn.proj", a)
        h = _lin(P, b + "mlp.fc2", F.gelu(_lin(P, b + "mlp.fc1", _ln(P, b + "norm2", t))))
        t = t + P[b + "ls2.gamma"] * h
        if i in idx:
            n = _ln(P, p + "norm", t)
            out.append((n[:, 1:], n[:, 0]))
        i += 1
    return out


# ----------------------------------------------------------------------------
# DPT head
# ----------------------------------------------------------------------------

def _rcu(P, name, x):
    """ResidualConvUnit (bn False), depth_anything/blocks.py:69-92."""
    y = _conv(P, name + ".conv1", F.relu(x), 1, 1)
    return _conv(P, name + ".conv2", F.relu(y), 1, 1) + x


def _ffb(P, name, *xs, size=None):
    """FeatureFusionBlock, depth_anything/blocks.py:126-153 (align_corners True)."""
    out = xs[0]
    if len(xs) == 2:
        out = out + _rcu(P, name + ".resConfUnit1", xs[1])
    out = _rcu(P, name + ".resConfUnit2", out)
    kw = {"scale_factor": 2} if size is None else {"size": tuple(size)}
    out = F.interpolate(out, **kw, mode="bilinear", align_corners=True)
    return _conv(P, name + ".out_conv", out)


def dpt_head(P: Params, p: str, feats, ph: int, pw: int, patch_size: int = 14):
    """DPTHead.forward(return_intermediate=True), depth_anything/dpt.py:105-142 ->
    (out, path_1, path_2, path_3, path_4, disp)."""
    layers = []
    for i, (x, _) in enumerate(feats):
        x = x.permute(0, 2, 1).reshape(x.shape[0], x.shape[-1], ph, pw)
        x = _conv(P, f"{p}projects.{i}", x)
        if i == 0:
            x = _deconv(P, f"{p}resize_layers.0", x, 4, 0)
        elif i == 1:
            x = _deconv(P, f"{p}resize_layers.1", x, 2, 0)
        elif i == 3:
            x = _conv(P, f"{p}resize_layers.3", x, 2, 1)
        layers.append(x)
    s = p + "scratch."
    rn = [_conv(P, f"{s}layer{i + 1}_rn", x, 1, 1) for i, x in enumerate(layers)]
    path_4 = _ffb(P, s + "refinenet4", rn[3], size=rn[2].shape[2:])
    path_3 = _ffb(P, s + "refinenet3", path_4, rn[2], size=rn[1].shape[2:])
    path_2 = _ffb(P, s + "refinenet2", path_3, rn[1], size=rn[0].shape[2:])
    path_1 = _ffb(P, s + "refinenet1", path_2, rn[0])
    out = _conv(P, s + "output_conv1", path_1, 1, 1)
    out = F.interpolate(out, (int(ph * patch_size), int(pw * patch_size)), mode="bilinear", align_corners=True)
    depth = F.relu(_conv(P, s + "output_conv2.0", out, 1, 1))
    depth = F.relu(F.relu(_conv(P, s + "output_conv2.2", depth)))
    disp = 1 / depth
    disp[depth == 0] = 0
    disp = disp / disp.max()
    return out, path_1, path_2, path_3, path_4, disp


def depth_anything_feature(P: Params, p: str, x: Tensor, encoder: str = "vits"):
    """DepthAnythingFeature.forward, core/extractor.py:308-320 -> dict."""
    _, _, heads = _VIT[encoder]
    feats = vit_intermediate(P, p + "depth_anything.pretrained.", x, _IDX[encoder], heads)
    ps = P[p + "depth_anything.pretrained.patch_embed.proj.weight"].shape[-1]
    h, w = x.shape[-2:]
    out, p1, p2, p3, p4, disp = dpt_head(P, p + "depth_anything.depth_head.", feats, h // ps, w // ps, ps)
    return {"out": out, "path_1": p1, "path_2": p2, "path_3": p3, "path_4": p4, "features": feats, "disp": disp}


# ----------------------------------------------------------------------------
# EdgeNeXt-S (timm edgenext_small, restated: parity unpinned against timm)
# ----------------------------------------------------------------------------

def _ln2d(P, name, x, eps=1e-6):
    """LayerNorm over channels of an NCHW map."""
    return F.layer_norm(x.permute(0, 2, 3, 1), (x.shape[1],), P[name + ".weight"], P[name + ".bias"],
                        eps).permute(0, 3, 1, 2)


def _mlp_tail(P, name, y, shortcut, gamma):
    """LayerNorm -> fc1 -> GELU -> fc2 -> gamma -> + shortcut on channels-last tokens."""
    t = y.permute(0, 2, 3, 1)
    t = _lin(P, name + ".mlp.fc2", F.gelu(_lin(P, name + ".mlp.fc1", _ln(P, name + ".norm", t))))
    return shortcut + (P[name + gamma] * t).permute(0, 3, 1, 2)


def _conv_block(P, name, x):
    """ConvBlock: depthwise k x k -> LN -> MLP -> gamma, + x."""
    k = P[name + ".conv_dw.weight"].shape[-1]
    y = _conv(P, name + ".conv_dw", x, 1, k // 2, groups=x.shape[1])
    return _mlp_tail(P, name, y, x, ".gamma")


def _fourier_pos(P, name, B, H, W, hidden=32, temperature=10000):
    """PositionalEncodingFourier (hidden 32): normalised cumulative y / x coordinates, sin / cos
    interleaved, 1x1 token projection."""
    y = torch.arange(1, H + 1, dtype=torch.float32).view(1, H, 1).expand(B, H, W)
    x = torch.arange(1, W + 1, dtype=torch.float32).view(1, 1, W).expand(B, H, W)
    y = y / (y[:, -1:, :] + 1e-6) * (2 * math.pi)
    x = x / (x[:, :, -1:] + 1e-6) * (2 * math.pi)
    dim_t = torch.arange(hidden, dtype=torch.float32)
    dim_t = temperature ** (2 * torch.div(dim_t, 2, rounding_mode="floor") / hidden)
    px, py = x[..., None] / dim_t, y[..., None] / dim_t
    px = torch.stack((px[..., 0::2].sin(), px[..., 1::2].cos()), dim=4).flatten(3)
    py = torch.stack((py[..., 0::2].sin(), py[..., 1::2].cos()), dim=4).flatten(3)
    pos = torch.cat((py, px), dim=3).permute(0, 3, 1, 2)
    return _conv(P, name + ".token_projection", pos)


def _split_transpose_block(P, name, x, heads=8):
    """SplitTransposeBlock: multi-scale depthwise split, cross-covariance attention, inverted bottleneck."""
    B, C, H, W = x.shape
    nconv = 0
    while f"{name}.convs.{nconv}.weight" in P:
        nconv += 1
    spx = x.chunk(nconv + 1, dim=1)
    spo = []
    sp = spx[0]
    for i in range(nconv):
        if i > 0:
            sp = sp + spx[i]
        sp = _conv(P, f"{name}.convs.{i}", sp, 1, 1, groups=sp.shape[1])
        spo.append(sp)
    spo.append(spx[-1])
    y = torch.cat(spo, 1)
    if name + ".pos_embd.token_projection.weight" in P:
        y = y + _fourier_pos(P, name + ".pos_embd", B, H, W)
    t = y.reshape(B, C, H * W).permute(0, 2, 1)                            # (B, N, C)
    n = _ln(P, name + ".norm_xca", t)
    qkv = _lin(P, name + ".xca.qkv", n).reshape(B, H * W, 3, heads, C // heads).permute(2, 0, 3, 4, 1)
    q, k, v = qkv[0], qkv[1], qkv[2]                                       # (B, heads, ch, N)
    q = q / q.norm(dim=-1, keepdim=True).clamp_min(1e-12)
    k = k / k.norm(dim=-1, keepdim=True).clamp_min(1e-12)
    a = torch.softmax((q @ k.transpose(-2, -1)) * P[name + ".xca.temperature"], -1)
    o = (a @ v).permute(0, 3, 1, 2).reshape(B, H * W, C)
    t = t + P[name + ".gamma_xca"] * _lin(P, name + ".xca.proj", o)
    y = t.permute(0, 2, 1).reshape(B, C, H, W)
    return _mlp_tail(P, name, y, x, ".gamma")


def edgenext_trunk(P: Params, p: str, x: Tensor) -> List[Tensor]:
    """stem + stages of edgenext_small -> [x4, x8, x16, x32] (core/extractor.py:358-362)."""
    y = _ln2d(P, p + "stem.1", _conv(P, p + "stem.0", x, 4, 0))
    outs = []
    for s in range(4):
        sp = f"{p}stages.{s}."
        if sp + "downsample.1.weight" in P:
            y = _conv(P, sp + "downsample.1", _ln2d(P, sp + "downsample.0", y), 2, 0)
        j = 0
        while f"{sp}blocks.{j}.mlp.fc1.weight" in P:
            b = f"{sp}blocks.{j}"
            y = _conv_block(P, b, y) if (b + ".conv_dw.weight") in P else _split_transpose_block(P, b, y)
            j += 1
        outs.append(y)
    return outs


# ----------------------------------------------------------------------------
# Feature
# ----------------------------------------------------------------------------

def resize_keep_aspect(H, W, divider=16, max_H=1232, max_W=1232):
    """get_resize_keep_aspect_ratio, Utils.py:89-105."""
    def rnd(x):
        return int(np.ceil(x / divider) * divider)
    Hr, Wr = rnd(H), rnd(W)
    if Hr > max_H or Wr > max_W:
        if Hr > Wr:
            Wr, Hr = rnd(Wr * max_H / Hr), max_H
        else:
            Hr, Wr = rnd(Hr * max_W / Wr), max_W
    return int(Hr), int(Wr)


def _resblock_in(P, name, x):
    """ResnetBasicBlock(norm_layer=InstanceNorm2d), core/submodule.py:119-156."""
    y = F.relu(_inorm(_conv(P, name + ".conv1", x, 1, 1)))
    return F.relu(_inorm(_conv(P, name + ".conv2", y, 1, 1)) + x)


def _conv2x_in(P, name, x, rem):
    """Conv2x_IN(deconv=True, concat=True), core/submodule.py:349-385."""
    x = _lrelu(_inorm(_deconv(P, name + ".conv1.conv", x, 2, 1)))
    if x.shape != rem.shape:
        x = F.interpolate(x, size=rem.shape[-2:], mode="bilinear")
    return _resblock_in(P, name + ".conv2", torch.cat([x, rem], 1))


def _residual_in(P, name, x):
    """ResidualBlock(norm_fn='instance', stride 1, same planes), core/extractor.py:20-80."""
    y = F.relu(_inorm(_conv(P, name + ".conv1", x, 1, 1)))
    y = F.relu(_inorm(_conv(P, name + ".conv2", y, 1, 1)))
    return F.relu(x + y)


def feature_forward(P: Params, p: str, x: Tensor, vit_size: str = "vits"):
    """Feature.forward, core/extractor.py:348-369: x (2B, 3, H, W) normalised images ->
    ([x4, x8, x16, x32], vit_feat)."""
    B, C, H, W = x.shape
    Hr, Wr = resize_keep_aspect(H, W, divider=int(np.lcm(14, 16)), max_H=1344, max_W=1344)
    x_in_ = F.interpolate(x, size=(Hr, Wr), mode="bicubic", align_corners=False)
    vit_feat = depth_anything_feature(P, p + "dino.", x_in_, vit_size)["out"]
    vit_feat = F.interpolate(vit_feat, size=(H // 4, W // 4), mode="bilinear", align_corners=True)
    x4, x8, x16, x32 = edgenext_trunk(P, p, x)
    x16 = _conv2x_in(P, p + "deconv32_16", x32, x16)
    x8 = _conv2x_in(P, p + "deconv16_8", x16, x8)
    x4 = _conv2x_in(P, p + "deconv8_4", x8, x4)
    x4 = torch.cat([x4, vit_feat], 1)
    x4 = _lrelu(_inorm(_conv(P, p + "conv4.0.conv", x4, 1, 1)))
    x4 = _residual_in(P, p + "conv4.1", x4)
    x4 = _residual_in(P, p + "conv4.2", x4)
    return [x4, x8, x16, x32], vit_feat
