"""Drop-in for ``core/utils/utils.py``: the caller-side shape contract and the sampler.

``InputPadder`` is pure host logic (replicate-pad to a multiple of
``divis_by``; split ``[wd//2, wd-wd//2, ht//2, ht-ht//2]`` in sintel mode).
``bilinear_sampler`` is the stereo (H == 1) specialisation of the reference
wrapper on the gfx950 sampler kernel, without the per-call ``unique()`` host
sync: the y coordinate is validated to be exactly zero only when
``check=True``.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import ops, torch_ops


class InputPadder:
    """core/utils/utils.py:17-41."""

    def __init__(self, dims, mode="sintel", divis_by=8, force_square=False):
        self.ht, self.wd = dims[-2:]
        if force_square:
            side = max(self.ht, self.wd)
            pad_ht = ((side // divis_by) + 1) * divis_by - self.ht
            pad_wd = ((side // divis_by) + 1) * divis_by - self.wd
        else:
            pad_ht = (-self.ht) % divis_by
            pad_wd = (-self.wd) % divis_by
        if mode == "sintel":
            self._pad = [pad_wd // 2, pad_wd - pad_wd // 2, pad_ht // 2, pad_ht - pad_ht // 2]
        else:
            self._pad = [pad_wd // 2, pad_wd - pad_wd // 2, 0, pad_ht]

    def pad(self, *inputs):
        assert all(x.ndim == 4 for x in inputs)
        return [F.pad(x, self._pad, mode="replicate") for x in inputs]

    def unpad(self, x):
        assert x.ndim == 4
        ht, wd = x.shape[-2:]
        return x[..., self._pad[2]:ht - self._pad[3], self._pad[0]:wd - self._pad[1]]


def bilinear_sampler(img, coords, mode="bilinear", mask=False, low_memory=False, check=False):
    """core/utils/utils.py:44-55 for img (P,C,1,Lx), coords (P,1,K,2) with y == 0."""
    H, W = img.shape[-2:]
    assert H == 1, "This is a stereo problem"
    if check:
        assert bool((coords[..., 1] == 0).all()), "This is a stereo problem"
    P = img.shape[0]
    dtype = img.dtype                    # the reference returns grid_sample's output in img.dtype
    x = coords[..., 0].reshape(P, -1).float()
    img = img.float()
    if torch_ops.available():
        out = torch_ops.op("bilinear_sampler_1d", img, x)(img, x)
    else:                                # same kernel over the ctypes front end (libfsmi.so alone)
        out = ops.bilinear_sampler_1d(img, x)
    out = out.reshape(P, img.shape[1], 1, -1).to(dtype)
    if mask:
        xg = 2 * x / (W - 1) - 1
        m = ((xg > -1) & (xg < 1)).float().reshape(tuple(coords.shape[:-1]) + (1,))
        return out, m
    return out


def coords_grid(batch, ht, wd):
    """core/utils/utils.py:58-61."""
    ys, xs = torch.meshgrid(torch.arange(ht), torch.arange(wd), indexing="ij")
    return torch.stack([xs, ys], dim=0).float()[None].repeat(batch, 1, 1, 1)
