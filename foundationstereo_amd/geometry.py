"""Drop-in for ``core/geometry.py``: the combined geometry encoding volume on HIP.

``Combined_Geo_Encoding_Volume(init_fmap1, init_fmap2, geo_volume, num_levels, dx)``
builds, once per pair, the all-pairs correlation pyramid (fp32 MFMA kernel
with the W2 avg-pool fused in its epilogue) and the D pyramid of the filtered
volume in its native (B,C,D,H,W) layout -- level 0 *is* the filtered volume,
no permute copy (core/geometry.py:29).  ``__call__(disp, coords)`` is one fused
lookup kernel per refinement iteration with no host synchronisation (the
reference's ``unique()`` assert in ``bilinear_sampler`` syncs 2L times per
iteration, core/utils/utils.py:49).
"""
from __future__ import annotations

import torch

from . import ops


class Combined_Geo_Encoding_Volume:
    def __init__(self, init_fmap1, init_fmap2, geo_volume, num_levels=2, dx=None, *, init_corr_pyramid=None):
        """core/geometry.py:9-40.  ``init_corr_pyramid``: the all-pairs pyramid of the same features,
        already computed (``corr_pyramid``; FoundationStereo.forward runs it right after the cost
        volume, alone on the chip, long before the filtered volume exists)."""
        self.num_levels = num_levels
        self.dx = dx
        self.radius = 4 if dx is None else (int(dx.numel()) - 1) // 2
        fl = init_fmap1.float()
        fr = init_fmap2.float()
        vol = geo_volume.float()
        B, C, D, H, W = vol.shape
        assert fl.shape[0] == B and fl.shape[2:] == (H, W), "feature / volume shape mismatch"
        # the reference's dx is linspace(-r, r, 2r+1) (core/foundation_stereo.py:179); the kernel
        # bakes that tap set in, so refuse anything else rather than silently diverge
        if dx is not None:
            ref = torch.linspace(-self.radius, self.radius, 2 * self.radius + 1)
            if not torch.equal(dx.detach().float().reshape(-1).cpu(), ref):
                raise ValueError("fsmi geo lookup supports dx = linspace(-r, r, 2r+1) only")
        if init_corr_pyramid is not None:
            assert len(init_corr_pyramid) == num_levels and init_corr_pyramid[0].shape == (B, H, W, W), \
                "init_corr_pyramid does not match the features"
            self.init_corr_pyramid = list(init_corr_pyramid)
        else:
            self.init_corr_pyramid = self.corr_pyramid(fl, fr, num_levels)
        self.geo_volume_pyramid = ops.volume_pyramid(vol, num_levels)
        self.shape = (B, C, D, H, W)

    def __call__(self, disp, coords=None, low_memory=False, out=None):
        """Per-iteration lookup (core/geometry.py:43-65).

        ``coords``: the left-image column of each pixel, any layout of B*H*W values (the reference's
        (B,H,W,1), core/foundation_stereo.py:231); the correlation taps sit at coords/2^i - disp/2^i + k
        exactly as the reference's ``init_x0`` (:57).  ``None`` -- what this package's forward passes --
        lets the kernel derive the column from the pixel index instead of loading it (the reference's
        own coords are that arange(W)).
        """
        if coords is not None:
            coords = coords.float()
        return ops.geo_lookup(self.geo_volume_pyramid, self.init_corr_pyramid, disp.float(), self.radius, out=out,
                              coords=coords)

    @staticmethod
    def corr_pyramid(fmap1, fmap2, num_levels):
        """core/geometry.py:24-40 on HIP: [(B,H,W,W>>i)], the avg-pool pyramid of ``corr``."""
        return ops.allpairs_corr(fmap1.float(), fmap2.float(), num_levels)

    @staticmethod
    def corr(fmap1, fmap2):
        """core/geometry.py:68-77 -> (B,H,W1,1,W2)."""
        B, D, H, W1 = fmap1.shape
        lv = ops.allpairs_corr(fmap1.float(), fmap2.float(), 1)[0]
        return lv.reshape(B, H, W1, 1, fmap2.shape[-1])
