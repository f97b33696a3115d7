"""Pipelined-staging halo tiles (cfg 32 + c, conv_halo.h conv_halo_pipe_kernel) vs the plain
register-weight tiles and fp64 torch.

The pipelined variant changes only WHEN a chunk is split and stored (inside the previous chunk's
MFMA stream, into the other LDS buffer): the products, their order and the block exponent are the
plain tile's, so its output must be bit-identical -- checked for every 2D register-weight tile (2..9, 11),
1x1 and 3x3, 1-3 input segments (one a channel slice), ragged rows / columns / couts / channel
chunks, split-K 1-3, the output-slice / gamma / residual epilogue, and an all-zero first chunk.
"""
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


@pytest.mark.parametrize("cfg", [2, 3, 4, 5, 6, 7, 8, 9, 11])
@pytest.mark.parametrize("k", [1, 3])
@pytest.mark.parametrize("nsplit", [1, 2, 3])
def test_pipe_bit_identical(ops_mod, cfg, k, nsplit):
    B, H, W = 2, 13, 45
    a_ = synth.normal(711, (B, 40, H, W))
    c_ = synth.normal(712, (B, 64, H, W))
    cout = 70
    w = synth.normal(713, (cout, 40 + 29, k, k), 0.2)
    bias = synth.normal(714, (cout,), 0.1)
    gamma = synth.uniform(715, (cout,), 0.5, 1.5)
    res = synth.normal(716, (B, cout + 6, H, W))
    segs = [g(a_), (g(c_), 7, 29)]
    pk = ops_mod.PackedConv(g(w), mode="halo")
    kw = dict(bias=g(bias), act="relu", gamma=g(gamma), nsplit=nsplit)
    out_p = torch.zeros(B, cout + 6, H, W, device=DEV)
    out_q = torch.zeros(B, cout + 6, H, W, device=DEV)
    ops_mod.conv2d(segs, pk, cfg=cfg, out=out_p, co0=3, res=g(res)[:, 3:3 + cout].contiguous(), **kw)
    ops_mod.conv2d(segs, pk, cfg=cfg + 32, out=out_q, co0=3, res=g(res)[:, 3:3 + cout].contiguous(), **kw)
    assert torch.equal(out_p, out_q), float((out_p - out_q).abs().max())
    x = torch.cat([t(a_), t(c_[:, 7:36])], 1).double()
    ref = F.relu(F.conv2d(x, t(w).double(), t(bias).double(), padding=k // 2)) * t(gamma).double().view(1, -1, 1, 1) \
        + t(res)[:, 3:3 + cout].double()
    err = float((out_q[:, 3:3 + cout].double().cpu() - ref).abs().max())
    assert err < 2e-5 + 1e-5 * float(ref.abs().max()), err
    assert not ops_mod.range_overflowed(reset=True)


@pytest.mark.parametrize("cfg", [3, 9, 11])
def test_pipe_zero_first_chunk(ops_mod, cfg):
    """Chunks 0 and 1 all zero: the exponent comes from chunk 2 (one extra block max + barrier)."""
    B, H, W = 1, 12, 40
    zero = torch.zeros(B, 64, H, W)
    x = torch.cat([zero, torch.randn(B, 64, H, W, generator=torch.Generator().manual_seed(3)) * 1e-5], 1)
    w = torch.randn(96, 128, 3, 3, generator=torch.Generator().manual_seed(4)) * 0.1
    pk = ops_mod.PackedConv(g(w), mode="halo")
    out = ops_mod.conv2d([x.to(DEV)], pk, cfg=cfg + 32, nsplit=1)
    plain = ops_mod.conv2d([x.to(DEV)], pk, cfg=cfg, nsplit=1)
    assert torch.equal(out, plain)
    ref = F.conv2d(x.double(), w.double(), padding=1)
    assert float((out.double().cpu() - ref).abs().max() / ref.abs().max()) < 3e-6


@pytest.mark.parametrize("k", [1, 3])
def test_tile11_safe_mode(ops_mod, k):
    """Safe range mode sends the 2D-only 5-row tile (cfg 11 / 43) to the volume instantiation of the
    4-row 256-cout tile: same conv within the split-precision tolerance."""
    B, H, W = 1, 15, 40
    x = torch.randn(B, 96, H, W, generator=torch.Generator().manual_seed(5))
    w = torch.randn(260, 96, k, k, generator=torch.Generator().manual_seed(6)) * 0.1
    pk = ops_mod.PackedConv(g(w), mode="halo")
    ref = F.conv2d(x.double(), w.double(), padding=k // 2)
    ops_mod.set_range_safe(True)
    try:
        outs = [ops_mod.conv2d([x.to(DEV)], pk, cfg=c, nsplit=1) for c in (11, 43)]
    finally:
        ops_mod.set_range_safe(False)
    for out in outs:
        assert float((out.double().cpu() - ref).abs().max() / ref.abs().max()) < 3e-6
