"""Drop-in for ``core/update.py``: the selective ConvGRU refinement block.

Convolutions run on MIOpen (``torch.nn``); everything between them that the
reference does as separate elementwise passes -- sigmoid of the z/r gates,
``r*h``, the ``cat([r*h, x])`` copy, ``tanh``, the ``(1-z)h + zq`` update and
the ``small*att + large*(1-att)`` selection -- is two fused gfx950 kernels per
SelectiveConvGRU (``ops.gru_reset``, ``ops.gru_blend``).  ``convz`` and
``convr`` of each GRU share their input, so they run as ONE convolution with
the two weight tensors stacked (half the passes over ``hx``).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from .submodule import EdgeNextConvEncoder

__all__ = ["DispHead", "ConvGRU", "BasicMotionEncoder", "pool2x", "pool4x", "interp", "RaftConvGRU",
           "SelectiveConvGRU", "BasicSelectiveMultiUpdateBlock"]


class DispHead(nn.Module):
    """core/update.py:20-32."""

    def __init__(self, input_dim=128, hidden_dim=256, output_dim=1):
        super().__init__()
        self.conv = nn.Sequential(
            nn.Conv2d(input_dim, input_dim, kernel_size=3, padding=1), nn.ReLU(),
            EdgeNextConvEncoder(input_dim, expan_ratio=4, kernel_size=7, norm=None),
            EdgeNextConvEncoder(input_dim, expan_ratio=4, kernel_size=7, norm=None),
            nn.Conv2d(input_dim, output_dim, 3, padding=1))

    def forward(self, x):
        return self.conv(x)


class ConvGRU(nn.Module):
    """core/update.py:34-48 (unused by FoundationStereo; kept for API parity)."""

    def __init__(self, hidden_dim, input_dim, kernel_size=3):
        super().__init__()
        p = kernel_size // 2
        self.convz = nn.Conv2d(hidden_dim + input_dim, hidden_dim, kernel_size, padding=p)
        self.convr = nn.Conv2d(hidden_dim + input_dim, hidden_dim, kernel_size, padding=p)
        self.convq = nn.Conv2d(hidden_dim + input_dim, hidden_dim, kernel_size, padding=p)

    def forward(self, h, cz, cr, cq, *x_list):
        x = torch.cat(x_list, dim=1)
        hx = torch.cat([h, x], dim=1)
        z = torch.sigmoid(self.convz(hx) + cz)
        r = torch.sigmoid(self.convr(hx) + cr)
        q = torch.tanh(self.convq(torch.cat([r * h, x], dim=1)) + cq)
        return (1 - z) * h + z * q


class BasicMotionEncoder(nn.Module):
    """core/update.py:51-70."""

    def __init__(self, args, ngroup=8):
        super().__init__()
        self.args = args
        cor_planes = args.corr_levels * (2 * args.corr_radius + 1) * (ngroup + 1)
        self.convc1 = nn.Conv2d(cor_planes, 256, 1, padding=0)
        self.convc2 = nn.Conv2d(256, 256, 3, padding=1)
        self.convd1 = nn.Conv2d(1, 64, 7, padding=3)
        self.convd2 = nn.Conv2d(64, 64, 3, padding=1)
        self.conv = nn.Conv2d(64 + 256, 128 - 1, 3, padding=1)

    def forward(self, disp, corr):
        cor = F.relu(self.convc2(F.relu(self.convc1(corr))))
        dsp = F.relu(self.convd2(F.relu(self.convd1(disp))))
        out = F.relu(self.conv(torch.cat([cor, dsp], dim=1)))
        return torch.cat([out, disp], dim=1)


def pool2x(x):
    return F.avg_pool2d(x, 3, stride=2, padding=1)


def pool4x(x):
    return F.avg_pool2d(x, 5, stride=4, padding=1)


def interp(x, dest):
    return F.interpolate(x, dest.shape[2:], mode="bilinear", align_corners=True)


def _stacked_zr(gru, cache):
    """[convz; convr] weights stacked along out-channels (cached per weight version)."""
    wz, wr, bz, br = gru.convz.weight, gru.convr.weight, gru.convz.bias, gru.convr.bias
    key = tuple((t.data_ptr(), t._version) for t in (wz, wr, bz, br))
    hit = cache.get(id(gru))
    if hit is None or hit[0] != key:
        with torch.no_grad():
            hit = (key, torch.cat([wz, wr], 0).contiguous(), torch.cat([bz, br], 0).contiguous())
        cache[id(gru)] = hit
    return hit[1], hit[2]


class RaftConvGRU(nn.Module):
    """core/update.py:83-95."""

    def __init__(self, hidden_dim=128, input_dim=256, kernel_size=3):
        super().__init__()
        p = kernel_size // 2
        self.convz = nn.Conv2d(hidden_dim + input_dim, hidden_dim, kernel_size, padding=p)
        self.convr = nn.Conv2d(hidden_dim + input_dim, hidden_dim, kernel_size, padding=p)
        self.convq = nn.Conv2d(hidden_dim + input_dim, hidden_dim, kernel_size, padding=p)
        self._zr_cache = {}

    def zr(self, hx):
        w, b = _stacked_zr(self, self._zr_cache)
        return F.conv2d(hx, w, b, padding=self.convz.padding)

    def forward(self, h, x, hx):
        zr = self.zr(hx)
        qin, _ = ops.gru_reset(zr, zr, h, x)
        q = self.convq(qin)
        ones = torch.ones_like(h[:, :1])
        return ops.gru_blend(zr, zr, q, q, h, ones)


class SelectiveConvGRU(nn.Module):
    """core/update.py:98-119 with fused gate kernels."""

    def __init__(self, hidden_dim=128, input_dim=256, small_kernel_size=1, large_kernel_size=3, patch_size=None):
        super().__init__()
        self.conv0 = nn.Sequential(nn.Conv2d(input_dim, input_dim, kernel_size=3, padding=1), nn.ReLU())
        self.conv1 = nn.Sequential(nn.Conv2d(input_dim + hidden_dim, input_dim + hidden_dim, kernel_size=3,
                                             padding=1), nn.ReLU())
        self.small_gru = RaftConvGRU(hidden_dim, input_dim, small_kernel_size)
        self.large_gru = RaftConvGRU(hidden_dim, input_dim, large_kernel_size)

    def forward(self, att, h, *x):
        x = torch.cat(x, dim=1) if len(x) > 1 else x[0]
        x = self.conv0(x)
        hx = self.conv1(torch.cat([x, h], dim=1))
        # .float(): no-ops in fp32; under the reference's fp16 autocast the gates stay fp32
        zr_s = self.small_gru.zr(hx).float()
        zr_l = self.large_gru.zr(hx).float()
        h = h.float()
        qs_in, ql_in = ops.gru_reset(zr_s, zr_l, h, x.float())
        q_s = self.small_gru.convq(qs_in).float()
        q_l = self.large_gru.convq(ql_in).float()
        return ops.gru_blend(zr_s, zr_l, q_s, q_l, h, att.float())


class BasicSelectiveMultiUpdateBlock(nn.Module):
    """core/update.py:122-159."""

    def __init__(self, args, hidden_dim=128, volume_dim=8):
        super().__init__()
        self.args = args
        self.encoder = BasicMotionEncoder(args, volume_dim)
        n = args.n_gru_layers
        if n == 3:
            self.gru16 = SelectiveConvGRU(hidden_dim, hidden_dim * 2)
        if n >= 2:
            self.gru08 = SelectiveConvGRU(hidden_dim, hidden_dim * (n == 3) + hidden_dim * 2)
        self.gru04 = SelectiveConvGRU(hidden_dim, hidden_dim * (n > 1) + hidden_dim * 2)
        self.disp_head = DispHead(hidden_dim, 256)
        self.mask = nn.Sequential(nn.Conv2d(128, 64, 3, padding=1), nn.ReLU(inplace=True),
                                  nn.Conv2d(64, 32, 3, padding=1), nn.ReLU(inplace=True))

    def forward(self, net, inp, corr, disp, att):
        n = self.args.n_gru_layers
        if n == 3:
            net[2] = self.gru16(att[2], net[2], inp[2], pool2x(net[1]))
        if n >= 2:
            if n > 2:
                net[1] = self.gru08(att[1], net[1], inp[1], pool2x(net[0]), interp(net[2], net[1]))
            else:
                net[1] = self.gru08(att[1], net[1], inp[1], pool2x(net[0]))
        motion = torch.cat([inp[0], self.encoder(disp, corr)], dim=1)
        if n > 1:
            net[0] = self.gru04(att[0], net[0], motion, interp(net[1], net[0]))
        delta_disp = self.disp_head(net[0])
        mask = .25 * self.mask(net[0])
        return net, mask, delta_disp
