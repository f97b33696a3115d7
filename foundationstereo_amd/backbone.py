"""The stereo backbone ``Feature`` on the HIP engine (core/extractor.py:286-369).

Module trees and ``state_dict`` keys are the reference's, so ``feature.*`` checkpoint keys load:

* ``DinoVisionTransformer`` -- the vendored DINOv2 ViT (dinov2/dinov2/models/vision_transformer.py,
  built as ``dinov2/dinov2/hub/backbones.py:18-61`` does: patch 14, image 518, LayerScale 1.0, no block
  chunks, no registers) with ``get_intermediate_layers``;
* ``DPTHead`` / ``DepthAnything`` (depth_anything/dpt.py:24-190, depth_anything/blocks.py) and
  ``DepthAnythingFeature`` (core/extractor.py:286-320);
* ``EdgeNeXt`` stem / stages restated from timm's published ``edgenext_small`` (core/extractor.py:327
  builds it with ``timm.create_model``; timm is not importable here, so this row is "parity unpinned"
  against timm);
* ``Feature`` (core/extractor.py:323-369).

Data path (CUDA tensors, inference): the ViT keeps its tokens channel-major, (B, C, Tp) with the N
patch tokens first, the class token at N and zero padding to Tp (a multiple of 64), so every Linear is
a 1x1 conv on the split-precision halo conv engine (``ops.conv2d`` over a (Tp/32) x 32 map) with its
bias, GELU, LayerScale and residual in the conv epilogue; LayerNorm, attention, patch assembly and the
resizes are csrc/backbone.hip kernels.  DPT and EdgeNeXt convs run on the same conv engine.  There is
no CPU path: CPU tensors raise (the CPU restatement is the test-only ``oracle``).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from . import submodule as _sub
from .extractor import DepthAnythingFeature as _DAFConfig, ResidualBlock
from .submodule import BasicConv, Conv2x_IN

__all__ = ["DinoVisionTransformer", "vit_small", "vit_base", "vit_large", "DPTHead", "DepthAnything",
           "DepthAnythingFeature", "EdgeNeXt", "edgenext_small", "Feature", "get_resize_keep_aspect_ratio"]


def _need_hip(x, what):
    if not (isinstance(x, torch.Tensor) and x.is_cuda):
        raise RuntimeError(f"{what}: the backbone runs on ROCm (HIP) device tensors only (CPU restatement: oracle/)")
    if torch.is_grad_enabled() and any(p.requires_grad for p in [x]):
        raise RuntimeError(f"{what}: inference-only (input requires grad)")


def _cached(mod, name, tensors, build):
    """``build()`` cached on ``mod`` until any tensor in ``tensors`` is replaced or modified."""
    key = tuple((t.data_ptr(), t._version) for t in tensors if t is not None)
    hit = mod.__dict__.get(name)
    if hit is None or hit[0] != key:
        with torch.no_grad():
            hit = (key, build())
        mod.__dict__[name] = hit
    return hit[1]


def _bias(b, n, dev):
    return b.detach().float().contiguous() if b is not None else torch.zeros(n, device=dev)


def _lin_pack(lin):
    """nn.Linear (out, in) -> (PackedConv as a 1x1 conv, bias)."""
    return _cached(lin, "_fsmi_lin", [lin.weight, lin.bias],
                   lambda: (ops.PackedConv(lin.weight.detach().float()[:, :, None, None]),
                            _bias(lin.bias, lin.out_features, lin.weight.device)))


def _conv_pack(conv):
    """nn.Conv2d (1x1 or 3x3, stride 1, 'same') -> (PackedConv, bias)."""
    return _cached(conv, "_fsmi_conv", [conv.weight, conv.bias],
                   lambda: (ops.PackedConv(conv.weight.detach().float()),
                            _bias(conv.bias, conv.out_channels, conv.weight.device)))


def _flat_pack(conv):
    """Conv2d with stride == kernel as a 1x1 conv over its space-to-depth input (channel (c*k+ky)*k+kx)."""
    return _cached(conv, "_fsmi_flat", [conv.weight, conv.bias],
                   lambda: (ops.PackedConv(conv.weight.detach().float().reshape(conv.out_channels, -1)[:, :, None, None]),
                            _bias(conv.bias, conv.out_channels, conv.weight.device)))


def _deconv_pack(deconv):
    """ConvTranspose2d with stride == kernel (k) as a 1x1 conv with k*k*Cout outputs, row (ky*k+kx)*Cout + co."""
    def build():
        w = deconv.weight.detach().float()                        # (Cin, Cout, k, k)
        cin, cout, k, _ = w.shape
        w1 = w.permute(2, 3, 1, 0).reshape(k * k * cout, cin)
        b = _bias(deconv.bias, cout, w.device).repeat(k * k)
        return ops.PackedConv(w1[:, :, None, None].contiguous()), b.contiguous()
    return _cached(deconv, "_fsmi_deconv", [deconv.weight, deconv.bias], build)


def _conv(conv, x, act=None, res=None, gamma=None, out=None):
    """Stride-1 'same' Conv2d on the halo engine with its bias, activation / LayerScale / residual."""
    pk, b = _conv_pack(conv)
    return ops.conv2d([x], pk, bias=b, act=act, gamma=gamma, res=res, out=out)


def _img(t, Tp):
    """(B, C, Tp) tokens as the (B, C, Tp/32, 32) map the conv engine tiles."""
    return t.view(t.shape[0], t.shape[1], Tp // 32, 32)


# ================================================================ DINOv2 ViT

class PatchEmbed(nn.Module):
    """dinov2/dinov2/layers/patch_embed.py:25-81 (norm = Identity)."""

    def __init__(self, img_size=224, patch_size=16, in_chans=3, embed_dim=768):
        super().__init__()
        self.img_size = (img_size, img_size)
        self.patch_size = (patch_size, patch_size)
        self.patches_resolution = (img_size // patch_size, img_size // patch_size)
        self.num_patches = self.patches_resolution[0] * self.patches_resolution[1]
        self.in_chans = in_chans
        self.embed_dim = embed_dim
        self.proj = nn.Conv2d(in_chans, embed_dim, kernel_size=patch_size, stride=patch_size)
        self.norm = nn.Identity()


class LayerScale(nn.Module):
    """dinov2/dinov2/layers/layer_scale.py (gamma)."""

    def __init__(self, dim, init_values=1e-5):
        super().__init__()
        self.gamma = nn.Parameter(init_values * torch.ones(dim))


class Mlp(nn.Module):
    """dinov2/dinov2/layers/mlp.py:16-40 (fc1 -> GELU -> fc2); timm's Mlp has the same keys."""

    def __init__(self, in_features, hidden_features, bias=True):
        super().__init__()
        self.fc1 = nn.Linear(in_features, hidden_features, bias=bias)
        self.act = nn.GELU()
        self.fc2 = nn.Linear(hidden_features, in_features, bias=bias)


class Attention(nn.Module):
    """dinov2/dinov2/layers/attention.py:36-99 (MemEffAttention without xformers = SDPA)."""

    def __init__(self, dim, num_heads=8, qkv_bias=True, proj_bias=True):
        super().__init__()
        self.dim = dim
        self.num_heads = num_heads
        self.scale = (dim // num_heads) ** -0.5
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.proj = nn.Linear(dim, dim, bias=proj_bias)


class Block(nn.Module):
    """dinov2/dinov2/layers/block.py:43-114 (eval: no drop path)."""

    def __init__(self, dim, num_heads, mlp_ratio=4.0, init_values=None):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim, eps=1e-6)
        self.attn = Attention(dim, num_heads=num_heads)
        self.ls1 = LayerScale(dim, init_values) if init_values else nn.Identity()
        self.norm2 = nn.LayerNorm(dim, eps=1e-6)
        self.mlp = Mlp(dim, int(dim * mlp_ratio))
        self.ls2 = LayerScale(dim, init_values) if init_values else nn.Identity()

    def run(self, x, T, Tp):
        """x (B, D, Tp) channel-major tokens, updated in place (both residual adds in conv epilogues)."""
        xi = _img(x, Tp)
        y = ops.channel_layernorm(x, self.norm1.weight, self.norm1.bias, self.norm1.eps)
        pk, b = _lin_pack(self.attn.qkv)
        qkv = ops.conv2d([_img(y, Tp)], pk, bias=b)
        a = ops.vit_attention(qkv, self.attn.num_heads, T, self.attn.scale)
        pk, b = _lin_pack(self.attn.proj)
        g1 = self.ls1.gamma if isinstance(self.ls1, LayerScale) else None
        ops.conv2d([_img(a, Tp)], pk, bias=b, gamma=None if g1 is None else g1.detach().float(), res=xi, out=xi)
        y = ops.channel_layernorm(x, self.norm2.weight, self.norm2.bias, self.norm2.eps, out=y)
        pk, b = _lin_pack(self.mlp.fc1)
        h = ops.conv2d([_img(y, Tp)], pk, bias=b, act="gelu")
        pk, b = _lin_pack(self.mlp.fc2)
        g2 = self.ls2.gamma if isinstance(self.ls2, LayerScale) else None
        ops.conv2d([h], pk, bias=b, gamma=None if g2 is None else g2.detach().float(), res=xi, out=xi)
        return x


class DinoVisionTransformer(nn.Module):
    """dinov2/dinov2/models/vision_transformer.py:45-330 (MLP FFN, no registers, block_chunks = 0)."""

    def __init__(self, img_size=518, patch_size=14, embed_dim=384, depth=12, num_heads=6, mlp_ratio=4.0,
                 init_values=1.0, interpolate_offset=0.1):
        super().__init__()
        self.num_features = self.embed_dim = embed_dim
        self.num_tokens = 1
        self.n_blocks = depth
        self.num_heads = num_heads
        self.patch_size = patch_size
        self.num_register_tokens = 0
        self.interpolate_antialias = False
        self.interpolate_offset = interpolate_offset
        self.patch_embed = PatchEmbed(img_size=img_size, patch_size=patch_size, in_chans=3, embed_dim=embed_dim)
        num_patches = self.patch_embed.num_patches
        self.cls_token = nn.Parameter(torch.zeros(1, 1, embed_dim))
        self.pos_embed = nn.Parameter(torch.zeros(1, num_patches + self.num_tokens, embed_dim))
        self.register_tokens = None
        self.chunked_blocks = False
        self.blocks = nn.ModuleList([Block(embed_dim, num_heads, mlp_ratio, init_values) for _ in range(depth)])
        self.norm = nn.LayerNorm(embed_dim, eps=1e-6)
        self.head = nn.Identity()
        self.mask_token = nn.Parameter(torch.zeros(1, embed_dim))

    # ---- position embedding table in the channel-major token order (weight preparation, per size)
    def _pos_table(self, ph, pw, Tp):
        def build():
            pos = self.pos_embed.detach().float()
            N0 = pos.shape[1] - 1
            M = int(math.sqrt(N0))
            assert N0 == M * M
            D = pos.shape[-1]
            if N0 == ph * pw and ph == pw:
                patch = pos[0, 1:]
            else:
                # interpolate_pos_encoding (vision_transformer.py:180-212): bicubic with the scale factors
                # (w0 + offset) / M, on the (1, D, M, M) grid
                sx = float(ph + self.interpolate_offset) / M
                sy = float(pw + self.interpolate_offset) / M
                g = F.interpolate(pos[0, 1:].reshape(1, M, M, D).permute(0, 3, 1, 2), mode="bicubic",
                                  antialias=self.interpolate_antialias, scale_factor=(sx, sy))
                assert tuple(g.shape[-2:]) == (ph, pw)
                patch = g[0].permute(1, 2, 0).reshape(ph * pw, D)
            tab = torch.zeros((D, Tp), device=pos.device, dtype=torch.float32)
            tab[:, :ph * pw] = patch.t()
            tab[:, ph * pw] = pos[0, 0]
            return tab.contiguous()
        return _cached(self, f"_fsmi_pos_{ph}_{pw}_{Tp}", [self.pos_embed], build)

    def prepare_tokens(self, x):
        """Patch embed + class token + position embedding -> ((B, D, Tp) tokens, N, Tp)
        (vision_transformer.py:214-233 in the channel-major layout)."""
        _need_hip(x, "DinoVisionTransformer")
        B, _, H, W = x.shape
        p = self.patch_size
        assert H % p == 0 and W % p == 0, f"input {H}x{W} is not a multiple of the patch size {p}"
        ph, pw = H // p, W // p
        N = ph * pw
        Tp = (N + 1 + 63) // 64 * 64
        pk, b = _flat_pack(self.patch_embed.proj)
        emb = ops.conv2d([ops.space_to_depth(x.float(), p)], pk, bias=b)      # (B, D, ph, pw)
        cls = self.cls_token.detach().float().reshape(-1)
        return ops.vit_tokens(emb, cls, self._pos_table(ph, pw, Tp), Tp), N, Tp

    def intermediate_maps(self, x, n, keep_states=True):
        """The normalised patch tokens after the blocks in ``n`` as (B, D, ph, pw) maps (plus, per block,
        the (B, D, Tp) token state for the class token when ``keep_states``), the HIP form of
        get_intermediate_layers."""
        B, _, H, W = x.shape
        ph, pw = H // self.patch_size, W // self.patch_size
        tok, N, Tp = self.prepare_tokens(x)
        take = range(len(self.blocks) - n, len(self.blocks)) if isinstance(n, int) else list(n)
        maps, states = [], []
        for i, blk in enumerate(self.blocks):
            blk.run(tok, N + 1, Tp)
            if i in take:
                m = ops.channel_layernorm(tok, self.norm.weight, self.norm.bias, self.norm.eps, n=N)
                maps.append(m.view(B, -1, ph, pw))
                if keep_states:
                    states.append(tok.clone() if i != len(self.blocks) - 1 else tok)
        assert len(maps) == len(take), f"only {len(maps)} / {len(take)} blocks found"
        return maps, states, N, Tp

    def get_intermediate_layers(self, x, n=1, reshape=False, return_class_token=False, norm=True):
        """vision_transformer.py:299-323: patch tokens (B, N, D) (or (B, D, h, w) with reshape) and class
        tokens (B, D)."""
        assert norm, "get_intermediate_layers: norm=False is not supported"
        maps, states, N, Tp = self.intermediate_maps(x, n)
        outs = [m if reshape else m.flatten(2).transpose(1, 2) for m in maps]
        if not return_class_token:
            return tuple(outs)
        cls = [ops.channel_layernorm(s, self.norm.weight, self.norm.bias, self.norm.eps, n=1, x_offset=N)[:, :, 0]
               for s in states]
        return tuple(zip(outs, cls))


def vit_small(patch_size=14, **kw):
    return DinoVisionTransformer(patch_size=patch_size, embed_dim=384, depth=12, num_heads=6, **kw)


def vit_base(patch_size=14, **kw):
    return DinoVisionTransformer(patch_size=patch_size, embed_dim=768, depth=12, num_heads=12, **kw)


def vit_large(patch_size=14, **kw):
    return DinoVisionTransformer(patch_size=patch_size, embed_dim=1024, depth=24, num_heads=16, **kw)


# ================================================================ DPT head

class ResidualConvUnit(nn.Module):
    """depth_anything/blocks.py:37-92 (bn False): conv2(relu(conv1(relu(x)))) + x."""

    def __init__(self, features, activation=None, bn=False):
        super().__init__()
        self.bn = bn
        self.groups = 1
        self.conv1 = nn.Conv2d(features, features, kernel_size=3, stride=1, padding=1, bias=True)
        self.conv2 = nn.Conv2d(features, features, kernel_size=3, stride=1, padding=1, bias=True)
        if bn:
            self.bn1 = nn.BatchNorm2d(features)
            self.bn2 = nn.BatchNorm2d(features)
        self.activation = nn.ReLU(False)

    def run(self, x, extra=None):
        """conv2(relu(conv1(relu(x)))) + x (+ extra, the fusion block's skip add)."""
        assert not self.bn, "DPT with use_bn is not supported on the HIP path"
        t = _conv(self.conv1, ops.elementwise(x, op="relu"), act="relu")
        return _conv(self.conv2, t, res=x if extra is None else ops.elementwise(x, extra, "add"))


class FeatureFusionBlock(nn.Module):
    """depth_anything/blocks.py:95-153 (deconv False, expand False, align_corners True)."""

    def __init__(self, features, bn=False, size=None):
        super().__init__()
        self.deconv = False
        self.align_corners = True
        self.groups = 1
        self.expand = False
        self.out_conv = nn.Conv2d(features, features, kernel_size=1, stride=1, padding=0, bias=True, groups=1)
        self.resConfUnit1 = ResidualConvUnit(features, None, bn)
        self.resConfUnit2 = ResidualConvUnit(features, None, bn)
        self.size = size

    def run(self, *xs, size=None):
        out = xs[0]
        if len(xs) == 2:
            out = self.resConfUnit1.run(xs[1], extra=out)       # out + resConfUnit1(xs[1])
        out = self.resConfUnit2.run(out)
        if size is None:
            size = self.size if self.size is not None else (2 * out.shape[-2], 2 * out.shape[-1])
        out = ops.resize_bilinear(out, tuple(int(s) for s in size))
        return _conv(self.out_conv, out)


class _Scratch(nn.Module):
    pass


class DPTHead(nn.Module):
    """depth_anything/dpt.py:24-146 (use_clstoken False)."""

    def __init__(self, nclass, in_channels, features=256, use_bn=False, out_channels=(256, 512, 1024, 1024),
                 use_clstoken=False):
        super().__init__()
        assert nclass == 1 and not use_clstoken, "DPTHead: the DepthAnythingFeature configuration (nclass 1, no cls)"
        self.nclass = nclass
        self.use_clstoken = use_clstoken
        oc = list(out_channels)
        self.projects = nn.ModuleList([nn.Conv2d(in_channels, c, kernel_size=1, stride=1, padding=0) for c in oc])
        self.resize_layers = nn.ModuleList([
            nn.ConvTranspose2d(oc[0], oc[0], kernel_size=4, stride=4, padding=0),
            nn.ConvTranspose2d(oc[1], oc[1], kernel_size=2, stride=2, padding=0),
            nn.Identity(),
            nn.Conv2d(oc[3], oc[3], kernel_size=3, stride=2, padding=1)])
        s = _Scratch()
        s.layer1_rn = nn.Conv2d(oc[0], features, kernel_size=3, stride=1, padding=1, bias=False)
        s.layer2_rn = nn.Conv2d(oc[1], features, kernel_size=3, stride=1, padding=1, bias=False)
        s.layer3_rn = nn.Conv2d(oc[2], features, kernel_size=3, stride=1, padding=1, bias=False)
        s.layer4_rn = nn.Conv2d(oc[3], features, kernel_size=3, stride=1, padding=1, bias=False)
        self.scratch = s
        s.stem_transpose = None
        s.refinenet1 = FeatureFusionBlock(features, use_bn)
        s.refinenet2 = FeatureFusionBlock(features, use_bn)
        s.refinenet3 = FeatureFusionBlock(features, use_bn)
        s.refinenet4 = FeatureFusionBlock(features, use_bn)
        s.output_conv1 = nn.Conv2d(features, features // 2, kernel_size=3, stride=1, padding=1)
        s.output_conv2 = nn.Sequential(nn.Conv2d(features // 2, 32, kernel_size=3, stride=1, padding=1), nn.ReLU(True),
                                       nn.Conv2d(32, 1, kernel_size=1, stride=1, padding=0), nn.ReLU(True),
                                       nn.Identity())

    def run(self, maps, patch_h, patch_w, patch_size=14, with_disp=True):
        """``maps``: the four normalised (B, D, ph, pw) token maps -> (out, path_1..path_4, disp or None)
        (dpt.py:105-142 with return_intermediate)."""
        layers = []
        for i, x in enumerate(maps):
            x = _conv(self.projects[i], x)
            r = self.resize_layers[i]
            if isinstance(r, nn.ConvTranspose2d):
                k = r.kernel_size[0]
                assert r.stride == (k, k) and r.padding == (0, 0) and r.kernel_size == (k, k)
                pk, b = _deconv_pack(r)
                x = ops.depth_to_space(ops.conv2d([x], pk, bias=b), k)
            elif isinstance(r, nn.Conv2d):
                x = _sub.conv2d_s2_bn_act(x, r, None)
            layers.append(x)
        s = self.scratch
        l1, l2, l3, l4 = (ops.conv2d([x], *_conv_pack(c)) for x, c in
                          zip(layers, (s.layer1_rn, s.layer2_rn, s.layer3_rn, s.layer4_rn)))
        path_4 = s.refinenet4.run(l4, size=l3.shape[2:])
        path_3 = s.refinenet3.run(path_4, l3, size=l2.shape[2:])
        path_2 = s.refinenet2.run(path_3, l2, size=l1.shape[2:])
        path_1 = s.refinenet1.run(path_2, l1)
        out = _conv(s.output_conv1, path_1)
        out = ops.resize_bilinear(out, (int(patch_h * patch_size), int(patch_w * patch_size)))
        disp = None
        if with_disp:
            c0, c2 = s.output_conv2[0], s.output_conv2[2]
            depth = _conv(c2, _conv(c0, out, act="relu"), act="relu")
            disp = torch.where(depth == 0, torch.zeros_like(depth), 1.0 / depth)
            disp = disp / disp.max()
        return out, path_1, path_2, path_3, path_4, disp


class DepthAnything(nn.Module):
    """DPT_DINOv2 / DepthAnything (depth_anything/dpt.py:149-190); ``pretrained`` is built locally the way
    dinov2/dinov2/hub/backbones.py:18-61 does (the reference fetches it with torch.hub, :159)."""

    def __init__(self, config):
        super().__init__()
        encoder = config["encoder"]
        assert encoder in ("vits", "vitb", "vitl")
        self.pretrained = {"vits": vit_small, "vitb": vit_base, "vitl": vit_large}[encoder]()
        dim = self.pretrained.blocks[0].attn.qkv.in_features
        self.depth_head = DPTHead(1, dim, config["features"], False, out_channels=config["out_channels"],
                                  use_clstoken=False)


class DepthAnythingFeature(nn.Module):
    """core/extractor.py:286-320."""
    model_configs = _DAFConfig.model_configs

    def __init__(self, encoder="vits"):
        super().__init__()
        self.encoder = encoder
        self.depth_anything = DepthAnything(self.model_configs[encoder])
        self.intermediate_layer_idx = {"vits": [2, 5, 8, 11], "vitb": [2, 5, 8, 11], "vitl": [4, 11, 17, 23],
                                       "vitg": [9, 19, 29, 39]}

    def forward(self, x, with_disp=True, with_features=True):
        """@x (B, 3, H, W) -> {'out', 'path_1'..'path_4', 'features', 'disp'} (core/extractor.py:308-320).
        ``with_disp`` / ``with_features`` False skip what Feature discards (the depth tail of the DPT
        head and the class tokens)."""
        _need_hip(x, "DepthAnythingFeature")
        h, w = x.shape[-2:]
        vit = self.depth_anything.pretrained
        maps, states, N, Tp = vit.intermediate_maps(x, self.intermediate_layer_idx[self.encoder],
                                                    keep_states=with_features)
        ph, pw = h // vit.patch_size, w // vit.patch_size
        out, p1, p2, p3, p4, disp = self.depth_anything.depth_head.run(maps, ph, pw, vit.patch_size,
                                                                       with_disp=with_disp)
        features = None
        if with_features:
            features = tuple((m.flatten(2).transpose(1, 2),
                              ops.channel_layernorm(s, vit.norm.weight, vit.norm.bias, vit.norm.eps, n=1,
                                                    x_offset=N)[:, :, 0]) for m, s in zip(maps, states))
        return {"out": out, "path_1": p1, "path_2": p2, "path_3": p3, "path_4": p4, "features": features,
                "disp": disp}


# ================================================================ EdgeNeXt-S (timm edgenext_small)

class LayerNorm2d(nn.LayerNorm):
    """timm LayerNorm2d (channels-first LayerNorm), eps 1e-6."""

    def __init__(self, num_channels, eps=1e-6):
        super().__init__(num_channels, eps=eps)

    def run(self, x):
        return ops.channel_layernorm(x, self.weight, self.bias, self.eps).view(x.shape)


class ConvBlock(nn.Module):
    """timm edgenext ConvBlock: dwconv k -> LayerNorm -> Linear 4C -> GELU -> Linear C -> gamma -> + x."""

    def __init__(self, dim, kernel_size=7, expand_ratio=4, ls_init_value=1e-6):
        super().__init__()
        self.shortcut_after_dw = False
        self.conv_dw = nn.Conv2d(dim, dim, kernel_size=kernel_size, padding=kernel_size // 2, groups=dim, bias=True)
        self.norm = nn.LayerNorm(dim, eps=1e-6)
        self.mlp = Mlp(dim, int(expand_ratio * dim))
        self.gamma = nn.Parameter(ls_init_value * torch.ones(dim)) if ls_init_value > 0 else None

    def run(self, x):
        y = ops.dwconv2d_ex(x, self.conv_dw.weight, self.conv_dw.bias)
        y = ops.channel_layernorm(y, self.norm.weight, self.norm.bias, self.norm.eps).view(x.shape)
        pk, b = _lin_pack(self.mlp.fc1)
        h = ops.conv2d([y], pk, bias=b, act="gelu")
        pk, b = _lin_pack(self.mlp.fc2)
        g = self.gamma.detach().float() if self.gamma is not None else None
        return ops.conv2d([h], pk, bias=b, gamma=g, res=x)


class PositionalEncodingFourier(nn.Module):
    """timm edgenext PositionalEncodingFourier (hidden 32, temperature 10000)."""

    def __init__(self, hidden_dim=32, dim=768, temperature=10000):
        super().__init__()
        self.token_projection = nn.Conv2d(hidden_dim * 2, dim, kernel_size=1)
        self.scale = 2 * math.pi
        self.hidden_dim = hidden_dim
        self.dim = dim
        self.temperature = temperature

    def table(self, H, W):
        """The (1, dim, H, W) embedding: a function of the map size and the projection weights only
        (weight preparation, cached per size)."""
        def build():
            dev = self.token_projection.weight.device
            y = torch.arange(1, H + 1, device=dev, dtype=torch.float32).view(1, H, 1).expand(1, H, W)
            x = torch.arange(1, W + 1, device=dev, dtype=torch.float32).view(1, 1, W).expand(1, H, W)
            eps = 1e-6
            y = y / (y[:, -1:, :] + eps) * self.scale
            x = x / (x[:, :, -1:] + eps) * self.scale
            dim_t = torch.arange(self.hidden_dim, dtype=torch.int64, device=dev).to(torch.float32)
            dim_t = self.temperature ** (2 * torch.div(dim_t, 2, rounding_mode="floor") / self.hidden_dim)
            px, py = x[..., None] / dim_t, y[..., None] / dim_t
            px = torch.stack((px[..., 0::2].sin(), px[..., 1::2].cos()), dim=4).flatten(3)
            py = torch.stack((py[..., 0::2].sin(), py[..., 1::2].cos()), dim=4).flatten(3)
            pos = torch.cat((py, px), dim=3).permute(0, 3, 1, 2)
            return F.conv2d(pos, self.token_projection.weight.float(), self.token_projection.bias.float()).contiguous()
        return _cached(self, f"_fsmi_pe_{H}_{W}", [self.token_projection.weight, self.token_projection.bias], build)


class CrossCovarianceAttn(nn.Module):
    """timm edgenext CrossCovarianceAttn (channel attention over tokens)."""

    def __init__(self, dim, num_heads=8, qkv_bias=True):
        super().__init__()
        self.num_heads = num_heads
        self.temperature = nn.Parameter(torch.ones(num_heads, 1, 1))
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.proj = nn.Linear(dim, dim)


class SplitTransposeBlock(nn.Module):
    """timm edgenext SplitTransposeBlock: multi-scale depthwise split, XCA, inverted bottleneck."""

    def __init__(self, dim, num_scales=1, num_heads=8, expand_ratio=4, use_pos_emb=True, ls_init_value=1e-6):
        super().__init__()
        width = max(int(math.ceil(dim / num_scales)), int(math.floor(dim // num_scales)))
        self.width = width
        self.num_scales = max(1, num_scales - 1)
        self.convs = nn.ModuleList([nn.Conv2d(width, width, kernel_size=3, padding=1, groups=width, bias=True)
                                    for _ in range(self.num_scales)])
        self.pos_embd = PositionalEncodingFourier(dim=dim) if use_pos_emb else None
        self.norm_xca = nn.LayerNorm(dim, eps=1e-6)
        self.gamma_xca = nn.Parameter(ls_init_value * torch.ones(dim)) if ls_init_value > 0 else None
        self.xca = CrossCovarianceAttn(dim, num_heads=num_heads, qkv_bias=True)
        self.norm = nn.LayerNorm(dim, eps=1e-6)
        self.mlp = Mlp(dim, int(expand_ratio * dim))
        self.gamma = nn.Parameter(ls_init_value * torch.ones(dim)) if ls_init_value > 0 else None

    def run(self, x):
        B, C, H, W = x.shape
        # x.chunk(len(convs) + 1, dim=1): pieces of ceil(C / n) channels, the last one shorter
        n = len(self.convs) + 1
        cs = -(-C // n)
        y = torch.empty_like(x)
        for i, conv in enumerate(self.convs):
            ops.dwconv2d_ex((x, i * cs, cs), conv.weight, conv.bias, add=None if i == 0 else (y, (i - 1) * cs, cs),
                            out=(y, i * cs, cs))
        y[:, (n - 1) * cs:] = x[:, (n - 1) * cs:]
        if self.pos_embd is not None:
            y = ops.elementwise(y, self.pos_embd.table(H, W), "add", broadcast=True)
        t = ops.channel_layernorm(y, self.norm_xca.weight, self.norm_xca.bias, self.norm_xca.eps).view(x.shape)
        pk, b = _lin_pack(self.xca.qkv)
        a = ops.xca(ops.conv2d([t], pk, bias=b), self.xca.temperature, self.xca.num_heads)
        pk, b = _lin_pack(self.xca.proj)
        g = self.gamma_xca.detach().float() if self.gamma_xca is not None else None
        y = ops.conv2d([a], pk, bias=b, gamma=g, res=y)
        t = ops.channel_layernorm(y, self.norm.weight, self.norm.bias, self.norm.eps).view(x.shape)
        pk, b = _lin_pack(self.mlp.fc1)
        h = ops.conv2d([t], pk, bias=b, act="gelu")
        pk, b = _lin_pack(self.mlp.fc2)
        g = self.gamma.detach().float() if self.gamma is not None else None
        return ops.conv2d([h], pk, bias=b, gamma=g, res=x)


class EdgeNeXtStage(nn.Module):
    """timm EdgeNeXtStage (downsample: LayerNorm2d + Conv2d k2 s2 when stride 2)."""

    def __init__(self, in_chs, out_chs, stride=2, depth=2, num_global_blocks=1, num_heads=4, scales=2,
                 kernel_size=7, expand_ratio=4, use_pos_emb=False, ls_init_value=1.0):
        super().__init__()
        if stride == 1:
            self.downsample = nn.Identity()
        else:
            self.downsample = nn.Sequential(LayerNorm2d(in_chs), nn.Conv2d(in_chs, out_chs, kernel_size=2, stride=2))
            in_chs = out_chs
        blocks = []
        for i in range(depth):
            if i < depth - num_global_blocks:
                blocks.append(ConvBlock(in_chs, kernel_size=kernel_size, expand_ratio=expand_ratio,
                                        ls_init_value=ls_init_value))
            else:
                blocks.append(SplitTransposeBlock(in_chs, num_scales=scales, num_heads=num_heads,
                                                  expand_ratio=expand_ratio, use_pos_emb=use_pos_emb,
                                                  ls_init_value=ls_init_value))
            in_chs = out_chs
        self.blocks = nn.Sequential(*blocks)

    def run(self, x):
        if not isinstance(self.downsample, nn.Identity):
            ln, conv = self.downsample
            pk, b = _flat_pack(conv)
            x = ops.conv2d([ops.space_to_depth(ln.run(x), conv.kernel_size[0])], pk, bias=b)
        for blk in self.blocks:
            x = blk.run(x)
        return x


class EdgeNeXt(nn.Module):
    """timm EdgeNeXt feature trunk (stem + stages; the head is not used by Feature)."""

    def __init__(self, dims=(24, 48, 88, 168), depths=(3, 3, 9, 3), global_block_counts=(0, 1, 1, 1),
                 kernel_sizes=(3, 5, 7, 9), heads=(8, 8, 8, 8), d2_scales=(2, 2, 3, 4),
                 use_pos_emb=(False, True, False, False), ls_init_value=1e-6, expand_ratio=4):
        super().__init__()
        self.stem = nn.Sequential(nn.Conv2d(3, dims[0], kernel_size=4, stride=4), LayerNorm2d(dims[0]))
        stages = []
        in_chs, stride_acc = dims[0], 4
        for i in range(4):
            stride = 2 if stride_acc == 2 or i > 0 else 1
            stride_acc *= stride
            stages.append(EdgeNeXtStage(in_chs, dims[i], stride=stride, depth=depths[i],
                                        num_global_blocks=global_block_counts[i], num_heads=heads[i],
                                        scales=d2_scales[i], kernel_size=kernel_sizes[i], expand_ratio=expand_ratio,
                                        use_pos_emb=use_pos_emb[i], ls_init_value=ls_init_value))
            in_chs = dims[i]
        self.stages = nn.Sequential(*stages)


def edgenext_small(**kw):
    """timm ``edgenext_small``: dims (48, 96, 160, 304), depths (3, 3, 9, 3)."""
    return EdgeNeXt(dims=(48, 96, 160, 304), depths=(3, 3, 9, 3), **kw)


def stem_run(stem, x):
    conv, ln = stem[0], stem[1]
    pk, b = _flat_pack(conv)
    return ln.run(ops.conv2d([ops.space_to_depth(x, conv.kernel_size[0])], pk, bias=b))


# ================================================================ Feature

def get_resize_keep_aspect_ratio(H, W, divider=16, max_H=1232, max_W=1232):
    """Utils.py:89-105."""
    assert max_H % divider == 0 and max_W % divider == 0

    def rnd(x):
        return int(np.ceil(x / divider) * divider)

    H_resize, W_resize = rnd(H), rnd(W)
    if H_resize > max_H or W_resize > max_W:
        if H_resize > W_resize:
            W_resize = rnd(W_resize * max_H / H_resize)
            H_resize = max_H
        else:
            H_resize = rnd(H_resize * max_W / W_resize)
            W_resize = max_W
    return int(H_resize), int(W_resize)


class Feature(nn.Module):
    """core/extractor.py:323-369: EdgeNeXt-S trunk + frozen DepthAnythingV2 features, fused at 1/4."""

    def __init__(self, args):
        super().__init__()
        self.args = args
        model = edgenext_small()
        self.stem = model.stem
        self.stages = model.stages
        chans = [48, 96, 160, 304]
        self.chans = chans
        self.dino = DepthAnythingFeature(encoder=self.args.vit_size).eval()
        for p in self.dino.parameters():
            p.requires_grad = False
        vit_feat_dim = DepthAnythingFeature.model_configs[self.args.vit_size]["features"] // 2
        self.deconv32_16 = Conv2x_IN(chans[3], chans[2], deconv=True, concat=True)
        self.deconv16_8 = Conv2x_IN(chans[2] * 2, chans[1], deconv=True, concat=True)
        self.deconv8_4 = Conv2x_IN(chans[1] * 2, chans[0], deconv=True, concat=True)
        c4 = chans[0] * 2 + vit_feat_dim
        self.conv4 = nn.Sequential(BasicConv(c4, c4, kernel_size=3, stride=1, padding=1, norm="instance"),
                                   ResidualBlock(c4, c4, norm_fn="instance"),
                                   ResidualBlock(c4, c4, norm_fn="instance"))
        self.patch_size = 14
        self.d_out = [chans[0] * 2 + vit_feat_dim, chans[1] * 2, chans[2] * 2, chans[3]]
        self.vit_dim = vit_feat_dim

    def forward(self, x):
        """x (2B, 3, H, W) normalised [left; right] images -> ([x4, x8, x16, x32], vit_feat)."""
        _need_hip(x, "Feature")
        x = x.float()
        B, C, H, W = x.shape
        divider = int(np.lcm(self.patch_size, 16))
        Hr, Wr = get_resize_keep_aspect_ratio(H, W, divider=divider, max_H=1344, max_W=1344)
        x_in_ = ops.resize_bicubic(x, (Hr, Wr))
        with torch.no_grad():
            vit_feat = self.dino(x_in_, with_disp=False, with_features=False)["out"]
        vit_feat = ops.resize_bilinear(vit_feat, (H // 4, W // 4))
        y = stem_run(self.stem, x)
        x4 = self.stages[0].run(y)
        x8 = self.stages[1].run(x4)
        x16 = self.stages[2].run(x8)
        x32 = self.stages[3].run(x16)
        x16 = self.deconv32_16(x32, x16)
        x8 = self.deconv16_8(x16, x8)
        x4 = self.deconv8_4(x8, x4)
        c = self.conv4[0]
        # cat([x4, vit_feat]) read in place as two segments of conv4[0]'s conv
        y = ops.instance_norm(_sub.conv2d_bn_act([x4, vit_feat], c.conv, None), act="leaky", eps=c.bn.eps)
        x4 = self.conv4[2](self.conv4[1](y))
        return [x4, x8, x16, x32], vit_feat
