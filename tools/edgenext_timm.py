"""Module-form restatement of timm's ``edgenext_small`` for the reference harness (build container only).

``core/extractor.py:327`` builds its EdgeNeXt-S trunk with ``timm.create_model('edgenext_small',
pretrained=True)``; timm is not installed here (no network), so ``tools/ref_harness.py`` answers that
call with this restatement of timm's published architecture: the product's module tree
(``foundationstereo_amd.backbone.edgenext_small``, timm's parameter names) with torch forwards written
the way timm's modules compute them (channels-last LayerNorm / MLP, ``x.chunk`` multi-scale split,
token-major cross-covariance attention).  Golden vectors of the reference ``Feature`` made with it pin
everything except the EdgeNeXt trunk itself, which stays "parity unpinned" against timm.

Never imported by the product, the GPU tests, ``smoke()`` or ``bench.py``.
"""
from __future__ import annotations

import math
import types

import torch
import torch.nn.functional as F


def _ln2d_forward(self, x):
    return F.layer_norm(x.permute(0, 2, 3, 1), self.normalized_shape, self.weight, self.bias,
                        self.eps).permute(0, 3, 1, 2)


def _mlp_forward(self, x):
    return self.fc2(self.act(self.fc1(x)))


def _conv_block_forward(self, x):
    shortcut = x
    x = self.conv_dw(x)
    x = x.permute(0, 2, 3, 1)
    x = self.norm(x)
    x = self.mlp(x)
    if self.gamma is not None:
        x = self.gamma * x
    x = x.permute(0, 3, 1, 2)
    return shortcut + x


def _pos_forward(self, B, H, W):
    dev = self.token_projection.weight.device
    inv_mask = ~torch.zeros((B, H, W), device=dev, dtype=torch.bool)
    y_embed = inv_mask.cumsum(1, dtype=torch.float32)
    x_embed = inv_mask.cumsum(2, dtype=torch.float32)
    eps = 1e-6
    y_embed = y_embed / (y_embed[:, -1:, :] + eps) * self.scale
    x_embed = x_embed / (x_embed[:, :, -1:] + eps) * self.scale
    dim_t = torch.arange(self.hidden_dim, dtype=torch.int64, device=dev).to(torch.float32)
    dim_t = self.temperature ** (2 * torch.div(dim_t, 2, rounding_mode="floor") / self.hidden_dim)
    pos_x = x_embed[:, :, :, None] / dim_t
    pos_y = y_embed[:, :, :, None] / dim_t
    pos_x = torch.stack((pos_x[:, :, :, 0::2].sin(), pos_x[:, :, :, 1::2].cos()), dim=4).flatten(3)
    pos_y = torch.stack((pos_y[:, :, :, 0::2].sin(), pos_y[:, :, :, 1::2].cos()), dim=4).flatten(3)
    pos = torch.cat((pos_y, pos_x), dim=3).permute(0, 3, 1, 2)
    return self.token_projection(pos)


def _xca_forward(self, x):
    B, N, C = x.shape
    qkv = self.qkv(x).reshape(B, N, 3, self.num_heads, -1).permute(2, 0, 3, 4, 1)
    q, k, v = qkv.unbind(0)
    attn = (F.normalize(q, dim=-1) @ F.normalize(k, dim=-1).transpose(-2, -1)) * self.temperature
    attn = attn.softmax(dim=-1)
    x = (attn @ v).permute(0, 3, 1, 2).reshape(B, N, C)
    return self.proj(x)


def _stb_forward(self, x):
    shortcut = x
    spx = x.chunk(len(self.convs) + 1, dim=1)
    spo = []
    sp = spx[0]
    for i, conv in enumerate(self.convs):
        if i > 0:
            sp = sp + spx[i]
        sp = conv(sp)
        spo.append(sp)
    spo.append(spx[-1])
    x = torch.cat(spo, 1)
    B, C, H, W = x.shape
    x = x.reshape(B, C, H * W).permute(0, 2, 1)
    if self.pos_embd is not None:
        x = x + self.pos_embd(B, H, W).reshape(B, -1, x.shape[1]).permute(0, 2, 1)
    x = x + self.gamma_xca * self.xca(self.norm_xca(x))
    x = x.reshape(B, H, W, C)
    x = self.norm(x)
    x = self.mlp(x)
    if self.gamma is not None:
        x = self.gamma * x
    x = x.permute(0, 3, 1, 2)
    return shortcut + x


def _stage_forward(self, x):
    return self.blocks(self.downsample(x))


def create_model(name, pretrained=False, features_only=False, **kw):
    """``timm.create_model`` stand-in: ``edgenext_small`` only, hash-initialised by the caller."""
    assert name == "edgenext_small", f"timm stub: {name} not restated"
    from foundationstereo_amd import backbone as bb
    m = bb.edgenext_small()
    table = {bb.LayerNorm2d: _ln2d_forward, bb.Mlp: _mlp_forward, bb.ConvBlock: _conv_block_forward,
             bb.PositionalEncodingFourier: _pos_forward, bb.CrossCovarianceAttn: _xca_forward,
             bb.SplitTransposeBlock: _stb_forward, bb.EdgeNeXtStage: _stage_forward}
    for mod in m.modules():
        fn = table.get(type(mod))
        if fn is not None:
            mod.forward = types.MethodType(fn, mod)
    return m
