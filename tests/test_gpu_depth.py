"""The depth-blocked (17, 1, 1) volume conv (cfg 30, csrc/conv_depth.hip) vs fp64 torch.

Conv3dNormActReduced.conv2 (core/submodule.py:89-114, kernel_disp = 17: hourglass conv1..3, agg_0,
agg_1, conv_out) is the disparity-axis conv; the tile walks each input plane once for 16 output
depths.  Covered: the hourglass channel counts (28 / 56 / 112 / 168: one to six 32-channel chunks,
one to six cout tiles), ragged channels / rows / columns, volumes shallower than the tile and than
the kernel, batch 2, ReLU / LeakyReLU / no activation, the FeatureAtt gate in the epilogue, planes
whose magnitudes differ by 1e11 (range mode 1: per-plane block exponent), and agreement with the
generic volume tile.  Tolerance 2e-5 abs + 1e-5 rel, as every split-precision volume conv.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from foundationstereo_amd import synth
from tests.helpers import t

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


def g(a):
    return t(a).to(DEV)


@pytest.fixture(scope="module")
def ops_mod():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from foundationstereo_amd import _lib, ops
    _lib.load()
    return ops


def close(a, b, atol=2e-5, rtol=1e-5):
    np.testing.assert_allclose(a.detach().double().cpu().numpy(), b.detach().double().cpu().numpy(),
                               atol=atol, rtol=rtol)


def _case(cin, cout, D, H, W, B, seed):
    gen = torch.Generator().manual_seed(seed)
    x = torch.randn(B, cin, D, H, W, generator=gen)
    w = torch.randn(cout, cin, 17, 1, 1, generator=gen) * 0.05
    bias = torch.randn(cout, generator=gen) * 0.1
    return x, w, bias


@pytest.mark.parametrize("act", ["relu", "leaky", None])
@pytest.mark.parametrize("cin,cout,D,H,W,B", [(28, 28, 48, 12, 40, 1), (56, 56, 24, 7, 33, 2),
                                              (112, 112, 12, 5, 20, 1), (168, 168, 6, 4, 10, 1),
                                              (28, 28, 5, 3, 40, 1), (40, 37, 20, 9, 70, 1)])
def test_depth_conv_vs_torch(ops_mod, cin, cout, D, H, W, B, act):
    x, w, bias = _case(cin, cout, D, H, W, B, cin + D + H)
    pk = ops_mod.PackedConv(g(w), mode="halo")
    out = ops_mod.conv3d(g(x), pk, bias=g(bias), act=act)          # auto: cfg 30
    ref = F.conv3d(x.double(), w.double(), bias.double(), padding=(8, 0, 0))
    if act == "relu":
        ref = F.relu(ref)
    elif act == "leaky":
        ref = F.leaky_relu(ref, 0.01)
    assert out.shape == ref.shape
    close(out, ref)
    # the generic volume tile computes the same conv
    gen = ops_mod.conv3d(g(x), pk, bias=g(bias), act=act, cfg=7, nsplit=1)
    close(out, gen)
    assert not ops_mod.range_overflowed(reset=True)


def test_depth_conv_feature_gate(ops_mod):
    """relu(conv + b) * sigmoid(gate) broadcast over depth (FeatureAtt in the epilogue)."""
    B, cin, cout, D, H, W = 2, 56, 56, 24, 9, 37
    x, w, bias = _case(cin, cout, D, H, W, B, 5)
    gate = torch.randn(B, cout, H, W, generator=torch.Generator().manual_seed(6)) * 3
    out = ops_mod.conv3d(g(x), ops_mod.PackedConv(g(w), mode="halo"), bias=g(bias), act="relu", fatt=g(gate))
    ref = F.relu(F.conv3d(x.double(), w.double(), bias.double(), padding=(8, 0, 0))) * \
        torch.sigmoid(gate.double()).unsqueeze(2)
    close(out, ref)


def test_depth_conv_plane_range(ops_mod):
    """Input planes spanning 1e-6 .. 1e5 (the bias-only w < d region of a cost volume next to
    correlation planes): the per-plane block exponent keeps the split's 22 bits relative to the
    output magnitude."""
    B, cin, cout, D, H, W = 1, 28, 28, 40, 6, 40
    x, w, bias = _case(cin, cout, D, H, W, B, 9)
    scale = torch.logspace(-6, 5, D).view(1, 1, D, 1, 1)
    x = x * scale
    out = ops_mod.conv3d(g(x), ops_mod.PackedConv(g(w), mode="halo"))
    ref = F.conv3d(x.double(), w.double(), padding=(8, 0, 0))
    assert bool(torch.isfinite(out).all())
    err = float((out.double().cpu() - ref).abs().max() / ref.abs().max())
    assert err < 3e-6, err
    # per output depth, relative to that depth's own magnitude (the window spans ~4 decades)
    rel = ((out.double().cpu() - ref).abs().amax((0, 1, 3, 4)) / ref.abs().amax((0, 1, 3, 4)))
    assert float(rel.max()) < 1e-4, rel


@pytest.mark.parametrize("cin,D,H,W,name", [(28, 48, 120, 160, "cfg2 conv_out / agg_0"),
                                            (56, 24, 60, 80, "cfg2 hourglass 1/8 (17,1,1)")])
def test_product_selects_depth_tile(ops_mod, cin, D, H, W, name):
    """What the product runs for cfg2's (17, 1, 1) convs: the tuning table's in-situ entry picks
    the depth tile (cfg 30) for these shapes, and the launch counters show conv_depth_kernel ran
    (not the generic volume tile) -- the same call path as Conv3dNormActReduced.conv2 (ops.conv3d,
    cfg / nsplit on auto).  Output agrees with the generic tile 7."""
    cfg, nsplit = ops_mod._tuned(1, 17, cin, cin, 1, D, H, W, -1, -1)
    assert (cfg, nsplit) == (30, 1), (name, cfg, nsplit)
    x, w, bias = _case(cin, cin, D, H, W, 1, cin + D)
    pk = ops_mod.PackedConv(g(w), mode="halo")
    ops_mod.conv_launch_counts(reset=True)
    out = ops_mod.conv3d(g(x), pk, bias=g(bias), act="relu")
    torch.cuda.synchronize()
    counts = ops_mod.conv_launch_counts(reset=True)
    assert counts[30] == 1 and sum(counts) == 1, [(i, c) for i, c in enumerate(counts) if c]
    generic = ops_mod.conv3d(g(x), pk, bias=g(bias), act="relu", cfg=7, nsplit=1)
    close(out, generic, atol=2e-5, rtol=1e-5)
