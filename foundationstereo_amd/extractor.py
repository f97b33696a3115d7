"""Context network and the backbone seam (``core/extractor.py``).

The context path runs once per pair before the refinement loop and is OUT of
the hot-path scope: it stays stock PyTorch-ROCm here, with
the reference's module tree so checkpoints load.  The backbone (EdgeNeXt-S +
DepthAnythingV2, ``Feature``) needs remote weights and is out of scope
(SURVEY §2 row 9); ``SyntheticFeature`` stands in for it, returning
device-resident feature maps with ``Feature.d_out`` channels.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops, synth
from .submodule import BasicConv, _fast2d, _fast_s2_2d, _hip_in, conv2d_bn_act, conv2d_s2_bn_act

__all__ = ["ResidualBlock", "ContextNetDino", "DepthAnythingFeature", "SyntheticFeature"]


class DepthAnythingFeature:
    """Only the config table of core/extractor.py:286-291 (the ViT itself is out of scope)."""
    model_configs = {
        "vitl": {"encoder": "vitl", "features": 256, "out_channels": [256, 512, 1024, 1024]},
        "vitb": {"encoder": "vitb", "features": 128, "out_channels": [96, 192, 384, 768]},
        "vits": {"encoder": "vits", "features": 64, "out_channels": [48, 96, 192, 384]},
    }


class ResidualBlock(nn.Module):
    """core/extractor.py:20-80 (batch / instance / none norms)."""

    def __init__(self, in_planes, planes, norm_fn="group", stride=1):
        super().__init__()
        self.conv1 = nn.Conv2d(in_planes, planes, kernel_size=3, padding=1, stride=stride)
        self.conv2 = nn.Conv2d(planes, planes, kernel_size=3, padding=1)
        self.relu = nn.ReLU(inplace=True)
        proj = not (stride == 1 and in_planes == planes)

        def mk():
            if norm_fn == "group":
                return nn.GroupNorm(num_groups=planes // 8, num_channels=planes)
            if norm_fn == "batch":
                return nn.BatchNorm2d(planes)
            if norm_fn == "instance":
                return nn.InstanceNorm2d(planes)
            return nn.Sequential()

        self.norm1 = mk()
        self.norm2 = mk()
        if proj:
            self.norm3 = mk()
        self.downsample = nn.Sequential(nn.Conv2d(in_planes, planes, kernel_size=1, stride=stride),
                                        self.norm3) if proj else None

    def forward(self, x):
        n1 = self.norm1 if isinstance(self.norm1, nn.BatchNorm2d) else None
        n2 = self.norm2 if isinstance(self.norm2, nn.BatchNorm2d) else None
        if n1 is not None and n2 is not None and _fast2d(x, self.conv2, n2):
            # every conv on the halo kernel with the eval BN folded in: stride-1 convs as 2D maps,
            # a downsampling block's 3x3 s2 conv and 1x1 s2 projection on the stride-2 tiles, the
            # projection finishing the block: relu(bn3(proj(x)) + y) in its epilogue
            if _fast2d(x, self.conv1, n1):
                y = conv2d_bn_act([x], self.conv1, n1, "relu")
            elif _fast_s2_2d(x, self.conv1, n1):
                y = conv2d_s2_bn_act(x, self.conv1, n1, "relu")
            else:
                y = F.relu(n1(self.conv1(x)))
            y = conv2d_bn_act([y], self.conv2, n2, "relu")
            if self.downsample is not None:
                pc, n3 = self.downsample
                if isinstance(n3, nn.BatchNorm2d) and _fast_s2_2d(x, pc, n3):
                    return conv2d_s2_bn_act(x, pc, n3, "relu", res=y, res_pre=True)
                x = self.downsample(x)
            return torch.relu_(y.add_(x))
        if (self.downsample is None and _hip_in(self.norm1, x) and _hip_in(self.norm2, x)
                and _fast2d(x, self.conv1, None) and _fast2d(x, self.conv2, None)):
            # norm_fn='instance' (Feature.conv4): relu(x + relu(IN(conv2(relu(IN(conv1 x))))))
            x = x.float()
            y = ops.instance_norm(conv2d_bn_act([x], self.conv1, None), act="relu", eps=self.norm1.eps)
            return ops.instance_norm(conv2d_bn_act([y], self.conv2, None), act="relu", res=x, act2="relu",
                                     eps=self.norm2.eps)
        y = F.relu(self.norm1(self.conv1(x)))
        y = F.relu(self.norm2(self.conv2(y)))
        if self.downsample is not None:
            x = self.downsample(x)
        return F.relu(x + y)


def _head(f, x):
    """Output head: [ResidualBlock,] Conv2d(3x3, bias); the conv on the halo kernel when it can."""
    if isinstance(f, nn.Conv2d):
        return conv2d_bn_act([x], f, None) if _fast2d(x, f, None) else f(x)
    x = f[0](x)
    return conv2d_bn_act([x], f[1], None) if _fast2d(x, f[1], None) else f[1](x)


class ContextNetDino(nn.Module):
    """core/extractor.py:192-283 (norm_fn='batch')."""

    def __init__(self, args, output_dim=[128], norm_fn="batch", downsample=3):
        super().__init__()
        self.args = args
        self.patch_size = 14
        self.image_size = 518
        self.vit_feat_dim = 384
        self.out_dims = output_dim
        self.norm_fn = norm_fn
        self.norm1 = nn.BatchNorm2d(64) if norm_fn == "batch" else nn.InstanceNorm2d(64)
        self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=1 + (downsample > 2), padding=3)
        self.relu1 = nn.ReLU(inplace=True)
        self.in_planes = 64
        self.layer1 = self._make_layer(64, stride=1)
        self.layer2 = self._make_layer(96, stride=1 + (downsample > 1))
        self.layer3 = self._make_layer(128, stride=1 + (downsample > 0))
        self.layer4 = self._make_layer(128, stride=2)
        self.layer5 = self._make_layer(128, stride=2)
        self.down = nn.Sequential(nn.Conv2d(128, 128, kernel_size=4, stride=4, padding=0), nn.BatchNorm2d(128))
        vit_dim = DepthAnythingFeature.model_configs[self.args.vit_size]["features"] // 2
        self.conv2 = BasicConv(128 + vit_dim, 128, kernel_size=3, padding=1)
        self.norm = nn.BatchNorm2d(256)
        self.outputs04 = nn.ModuleList([nn.Sequential(ResidualBlock(128, 128, norm_fn, stride=1),
                                                      nn.Conv2d(128, d[2], 3, padding=1)) for d in output_dim])
        self.outputs08 = nn.ModuleList([nn.Sequential(ResidualBlock(128, 128, norm_fn, stride=1),
                                                      nn.Conv2d(128, d[1], 3, padding=1)) for d in output_dim])
        self.outputs16 = nn.ModuleList([nn.Conv2d(128, d[0], 3, padding=1) for d in output_dim])

    def _make_layer(self, dim, stride=1):
        layers = nn.Sequential(ResidualBlock(self.in_planes, dim, self.norm_fn, stride=stride),
                               ResidualBlock(dim, dim, self.norm_fn, stride=1))
        self.in_planes = dim
        return layers

    def forward(self, x_in, vit_feat, dual_inp=False, num_layers=3):
        x = self.relu1(self.norm1(self.conv1(x_in)))
        x = self.layer3(self.layer2(self.layer1(x)))
        if _fast2d(x, self.conv2.conv, self.conv2.bn) and vit_feat.is_contiguous() and x.shape[1] % 8 == 0:
            x = conv2d_bn_act([x, vit_feat], self.conv2.conv, self.conv2.bn, "leaky")   # cat as segments
        else:
            x = self.conv2(torch.cat([x, vit_feat], dim=1))
        o4 = [_head(f, x) for f in self.outputs04]
        y = self.layer4(x)
        o8 = [_head(f, y) for f in self.outputs08]
        z = self.layer5(y)
        o16 = [_head(f, z) for f in self.outputs16]
        return o4, o8, o16


class SyntheticFeature(nn.Module):
    """Stand-in for ``Feature`` (core/extractor.py:323-369).

    ``set_features(left, right, vit)`` installs device-resident feature maps
    (the backbone output, already in HBM); ``forward`` returns them in the
    reference's ``([x4, x8, x16, x32], vit_feat)`` form for the concatenated
    ``[left; right]`` batch.  Without installed features it synthesises them
    from ``synth.backbone_features`` for the image size (host-side; tests).
    """

    def __init__(self, args):
        super().__init__()
        self.args = args
        self.d_out, self.vit_dim = synth.feature_dims(args.vit_size)
        self._preset = None
        self._by_size = {}         # (H, W) of the input images -> preset (hierarchical passes)
        self.shift_px = 0          # right-map shift of the synthesised features (no preset)

    def set_features(self, left, right, vit, size=None):
        """Install device-resident features; with ``size=(H, W)`` only for inputs of that image
        size (the two passes of run_hierachical see two sizes)."""
        if size is None:
            self._preset = (list(left), list(right), vit)
        else:
            self._by_size[tuple(size)] = (list(left), list(right), vit)

    def forward(self, x):
        hit = self._by_size.get(tuple(x.shape[-2:]))
        if hit is not None:
            left, right, vit = hit
        elif self._preset is None:
            B2, _, H, W = x.shape
            fl, fr, vit = synth.backbone_features(B2 // 2, H, W, self.args.vit_size, shift_px=self.shift_px)
            left = [torch.from_numpy(a).to(x.device) for a in fl]
            right = [torch.from_numpy(a).to(x.device) for a in fr]
            vit = torch.from_numpy(vit).to(x.device)
        else:
            left, right, vit = self._preset
        out = [torch.cat([a, b], 0) for a, b in zip(left, right)]
        return out, torch.cat([vit, vit], 0)
