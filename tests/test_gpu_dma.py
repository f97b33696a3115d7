"""Regression test for the pointwise tiles' LDS-DMA ring (csrc/conv_pw.hip dma16).

Round 4 found the DMA's inline asm writing M0 without saving it (the compiler keeps its own value
there) and without the one wait state an M0 write needs before an LDS-DMA: a DMA occasionally used a
stale M0 and filled another ring slot, and about 1 in 40 runs of the split-K pointwise tests saw
wrong partial sums (an eighth of the pixel tiles off).  Here every pointwise tile runs the same
split-K conv many times back to back; all repetitions must be bit-identical and match fp64 torch.
"""
import pytest
import torch
import torch.nn.functional as F

from foundationstereo_amd import synth

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module")
def ops_mod():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from foundationstereo_amd import _lib, ops
    _lib.load()
    return ops


@pytest.mark.parametrize("cfg", [24, 25, 26, 27, 28, 29])
@pytest.mark.parametrize("nsplit", [1, 2, 3])
def test_pw_dma_repeatable(ops_mod, cfg, nsplit):
    B, cin, cout, H, W = 2, 96, 130, 16, 40
    x = torch.from_numpy(synth.normal(881, (B, cin, H, W)))
    w = torch.from_numpy(synth.normal(882, (cout, cin, 1, 1), 0.2))
    pk = ops_mod.PackedConv(w.to(DEV), mode="halo")
    xg = x.to(DEV)
    with torch.no_grad():
        outs = [ops_mod.conv2d([xg], pk, cfg=cfg, nsplit=nsplit) for _ in range(24)]
    torch.cuda.synchronize()
    first = outs[0]
    for o in outs[1:]:
        assert torch.equal(o, first)
    ref = F.conv2d(x.double(), w.double())
    assert float((first.double().cpu() - ref).abs().max() / ref.abs().max()) < 3e-6
