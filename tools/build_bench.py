#!/usr/bin/env python3
"""Time the fused cost-volume build (gwc + concat + corr_stem[0]) over tile shapes.

    python tools/build_bench.py [--config cfg2] [--tiles 16,12 8,12 ...] [--reps 50]

Per variant: mean us over `reps` launches (HIP events on the launch stream), the
algorithmic bytes (bench.build_bytes: features + A/Bm read, Cs-channel volume
written) and GB/s; every variant is checked against the two-pass path.
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from foundationstereo_amd import ops  # noqa: E402

CFG = {"cfg1": (256, 320, 64, 128), "cfg2": (480, 640, 192, 128), "cfg2l": (480, 640, 192, 224),
       "cfg4": (384, 1248, 256, 224), "cfg5": (1024, 1536, 320, 224)}

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="cfg2")
ap.add_argument("--reps", type=int, default=50)
ap.add_argument("--dbg", type=int, nargs="*", default=[0], help="FSMI_BUILD_DBG values (1 no dots, 2 no stores)")
ap.add_argument("--tiles", nargs="*", default=["", "16,12", "8,12", "16,6", "8,6", "4,12", "16,16", "8,16"])
a = ap.parse_args()
H, W, md, C = CFG[a.config]
H4, W4, D4 = H // 4, W // 4, md // 4
Cs, G = 28, 8
dev = torch.device("cuda:0")
gen = torch.Generator(device=dev).manual_seed(0)
fl = torch.randn(1, C, H4, W4, device=dev, generator=gen)
fr = torch.randn(1, C, H4, W4, device=dev, generator=gen)
A = torch.randn(1, Cs, H4, W4, device=dev, generator=gen)
Bm = torch.randn(1, Cs, H4, W4, device=dev, generator=gen)
Wg = torch.randn(Cs, G, device=dev, generator=gen) * 0.3
nbytes = 4 * H4 * W4 * (2 * C + 2 * Cs + Cs * D4)


def timeit(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / a.reps


ref = ops.comb_volume_stem(fl, fr, A, Bm, Wg, D4, two_pass=True)
us = timeit(lambda: ops.comb_volume_stem(fl, fr, A, Bm, Wg, D4, two_pass=True))
print(f"{a.config} C={C} {H4}x{W4} D4={D4}: {nbytes / 1e6:.1f} MB algorithmic")
print(f"  two-pass            {us:8.1f} us  {nbytes / us / 1e3:7.0f} GB/s")
vol = torch.empty_like(ref)
us = timeit(lambda: vol.fill_(1.0))
print(f"  torch fill_ (same volume)  {us:8.1f} us  {vol.numel() * 4 / us / 1e3:7.0f} GB/s written")
for dbg in a.dbg:
    os.environ["FSMI_BUILD_DBG"] = str(dbg)
    for tile in a.tiles:
        os.environ["FSMI_BUILD_TILE"] = tile
        out = ops.comb_volume_stem(fl, fr, A, Bm, Wg, D4)
        err = float((out - ref).abs().max())
        us = timeit(lambda: ops.comb_volume_stem(fl, fr, A, Bm, Wg, D4))
        print(f"  one-pass dbg{dbg} {tile or 'auto':>8}  {us:8.1f} us  {nbytes / us / 1e3:7.0f} GB/s  max|diff| {err:.1e}")
os.environ.pop("FSMI_BUILD_TILE", None)
os.environ.pop("FSMI_BUILD_DBG", None)
