"""Range guard of the split-precision convs, enforced (round 3).

The split (fp16 hi + lo, ~22 bits) keeps its precision only inside fp16's range after a block
exponent.  2D convs fix that exponent from the first 32-channel chunk holding a nonzero value
(range mode 2, 8 bits of headroom); a later value beyond the headroom raises the range flag.
These tests check that no path returns a result computed past the flag:

* safe range mode (``ops.set_range_safe``): 2D convs on the per-chunk exponent (mode 1, the
  volumes' mode) -- an input whose second chunk is 1e7 x the first is exact to the split's
  precision and leaves the flag clear, on every tile family incl. the pointwise tiles;
* an all-zero first chunk no longer fixes scale 1 (small later values kept at ~22 bits);
* ``FoundationStereo.forward`` with an activation layout that overflows mode 2 (a function-
  preserving 2^-14 / 2^14 rescale of gru04.conv0's first input segment): the forward notices the
  flag, re-runs in safe mode and matches the CPU oracle of the unscaled model (< 1e-3 px);
* the same through ``ShardedStereo``'s captured hipGraph (replay -> flag -> eager safe re-run ->
  re-capture), at world size 1.
"""
import numpy as np
import pytest
import torch

import oracle
from foundationstereo_amd import ops, synth
from tests.helpers import load_golden, t

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


def g(a):
    return t(a).to(DEV)


@pytest.fixture
def lib():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from foundationstereo_amd import _lib
    _lib.load()
    ops.set_range_safe(False)
    ops.range_overflowed(reset=True)
    yield
    ops.set_range_safe(False)          # sticky: never leak safe mode into other tests
    ops.range_overflowed(reset=True)


def _rel_err(out, ref):
    return float((out.double().cpu() - ref).abs().max() / ref.abs().max())


@pytest.mark.parametrize("cfg", [-1, 1, 3, 4, 9, 19, 24, 25, 26, 27, 28, 29])
@pytest.mark.parametrize("k", [1, 3])
def test_safe_mode_conv2d(lib, cfg, k):
    """[small chunk, chunk 1e7 x larger]: mode 2 flags it; safe mode computes it to ~22 bits."""
    import torch.nn.functional as F
    if cfg >= 24 and k != 1:
        pytest.skip("pointwise tiles are 1x1")
    B, H, W = 1, 12, 40
    small = synth.normal(481, (B, 32, H, W)) * 1e-3
    big = synth.normal(482, (B, 40, H, W)) * 1e4
    w = synth.normal(483, (64, 72, k, k), 0.2)
    pk = ops.PackedConv(g(w), mode="halo")
    ref = F.conv2d(torch.cat([t(small), t(big)], 1).double(), t(w).double(), padding=k // 2)
    ops.conv2d([g(small), g(big)], pk, cfg=cfg, nsplit=1)
    assert ops.range_overflowed(reset=True), "mode 2 should flag a chunk 1e7 x its first"
    ops.set_range_safe(True)
    for nsplit in (1, 2):
        out = ops.conv2d([g(small), g(big)], pk, cfg=cfg, nsplit=nsplit)
        assert bool(torch.isfinite(out).all())
        err = _rel_err(out, ref)
        assert err < 3e-6, (nsplit, err)
    assert not ops.range_overflowed(reset=True)


@pytest.mark.parametrize("cfg", [-1, 3, 9, 19, 24])
def test_zero_first_chunk(lib, cfg):
    """An all-zero first chunk (dead ReLU channels) defers the exponent to the first nonzero chunk:
    later values ~1e-5 (fp16 subnormal at scale 1) keep the split's precision."""
    import torch.nn.functional as F
    k = 1 if cfg >= 24 else 3
    B, H, W = 1, 12, 40
    zero = np.zeros((B, 32, H, W), np.float32)
    tiny = synth.normal(484, (B, 32, H, W)) * 1e-5
    w = synth.normal(485, (48, 64, k, k), 0.2)
    ref = F.conv2d(torch.cat([t(zero), t(tiny)], 1).double(), t(w).double(), padding=k // 2)
    out = ops.conv2d([g(zero), g(tiny)], ops.PackedConv(g(w), mode="halo"), cfg=cfg, nsplit=1)
    assert _rel_err(out, ref) < 3e-6
    assert not ops.range_overflowed(reset=True)


H, W, MD, ITERS, L, SHIFT = 64, 96, 32, 4, 2, 2
SCALE = 2.0 ** 14


def _overflowing_model(args):
    """The tiny smoke model with gru04.conv0's first input segment (inp[0], 128 channels) scaled by
    2^-14 and the matching weight columns by 2^14: the same function (exact powers of two), but
    the conv's first chunk is now ~2^14 below the motion features that follow it -- beyond mode
    2's 2^9 headroom.  (2^14 keeps the conv's packed weight rows inside the split's range: a row is
    scaled by one exponent per output channel, and columns 2^20 apart would push the small ones'
    lo halves below fp16's normal range -- a weight span no checkpoint has.)"""
    from foundationstereo_amd.foundation_stereo import FoundationStereo
    m = FoundationStereo(args).eval()
    synth.init_module_(m, seed=1234)
    m = m.to(DEV)
    P = {k: v.detach().float().cpu() for k, v in m.state_dict().items()}
    conv0 = m.update_block.gru04.conv0[0]
    with torch.no_grad():
        conv0.weight[:, :128].mul_(SCALE)
    ctx = m._context

    def scaled_context(image1, vit_feat):
        stem_2x, net_list, inp_list, att = ctx(image1, vit_feat)
        return stem_2x, net_list, [inp_list[0] / SCALE] + list(inp_list[1:]), att
    m._context = scaled_context
    fl, fr, vf = synth.backbone_features(1, H, W, "vits", shift_px=SHIFT)
    m.feature.set_features([g(a) for a in fl], [g(a) for a in fr], g(vf))
    left, right = synth.stereo_images(1, H, W)
    with torch.no_grad():
        ref = oracle.oracle_forward(P, args, t(left), t(right), [t(a) for a in fl], [t(a) for a in fr], t(vf),
                                    iters=ITERS)
    return m, g(left), g(right), ref


@pytest.fixture
def no_split(monkeypatch):
    # split-K can put inp[0]'s chunks and the motion chunks in different blocks (each split takes
    # its own first-chunk exponent); one split per conv makes the overflow certain
    monkeypatch.setattr(ops, "_SPLIT_MAXPIX", 10 ** 9)
    # the trigger is a small FIRST segment of gru04.conv0 (inp[0]); with the context part hoisted
    # (update.CTX_PRE) inp[0] is convolved alone, uniformly scaled, and cannot overflow -- these tests
    # exercise the guard / recovery machinery, so they run conv0 whole
    from foundationstereo_amd import update
    monkeypatch.setattr(update, "CTX_PRE", False)


def test_forward_recovers_from_overflow(lib, no_split):
    args = synth.make_args(max_disp=MD, corr_levels=L, vit_size="vits")
    m, left, right, ref = _overflowing_model(args)
    n0 = ops.RANGE_RECOVERIES[0]
    with torch.no_grad():
        out = m(left, right, iters=ITERS, test_mode=True)
    assert ops.RANGE_RECOVERIES[0] == n0 + 1, "the overflow was not detected"
    assert ops.range_safe()
    d = float((out.cpu() - ref).abs().max())
    assert d < 1e-3, d
    # golden of the unscaled model: the same function
    d_gold = float(np.abs(out.cpu().numpy() - load_golden("e2e_tiny")["disp"]).max())
    assert d_gold < 1e-3, d_gold
    # guard off: the mode-2 result is what the guard prevents from being returned silently
    ops.set_range_safe(False)
    import foundationstereo_amd.foundation_stereo as fs
    fs.RANGE_GUARD = False
    try:
        with torch.no_grad():
            m(left, right, iters=ITERS, test_mode=True)
        assert ops.range_overflowed(reset=True)
    finally:
        fs.RANGE_GUARD = True


def test_sharded_replay_recovers_from_overflow(lib, no_split):
    from foundationstereo_amd.dist import ShardedStereo
    args = synth.make_args(max_disp=MD, corr_levels=L, vit_size="vits")
    m, left, right, ref = _overflowing_model(args)

    def fn(a, b):
        return m(a, b, iters=ITERS, test_mode=True)
    sh = ShardedStereo(fn, 0, 1)
    batch = torch.stack([left, right], 1)
    import foundationstereo_amd.foundation_stereo as fs
    fs.RANGE_GUARD = False                       # warm up + capture in mode 2 (the overflowing graph)
    try:
        with torch.no_grad():
            sh.step(batch, (1, H, W))
            ops.range_overflowed(reset=True)
            sh.capture(batch)
    finally:
        fs.RANGE_GUARD = True
    n0 = ops.RANGE_RECOVERIES[0]
    with torch.no_grad():
        out1 = sh.step(batch, (1, H, W)).clone()
        out2 = sh.step(batch, (1, H, W)).clone()      # the re-captured safe-mode graph
    assert ops.RANGE_RECOVERIES[0] == n0 + 1
    for out in (out1, out2):
        d = float((out.cpu() - ref).abs().max())
        assert d < 1e-3, d


def test_captured_forward_poisons_on_overflow(lib, no_split):
    """Without the per-replay host check (ShardedStereo.recover = False: no synchronisation), a
    replay whose convs overflowed returns NaN -- the captured forward's last node fills it -- and
    leaves the flag set for ops.check_range()."""
    from foundationstereo_amd.dist import ShardedStereo
    args = synth.make_args(max_disp=MD, corr_levels=L, vit_size="vits")
    m, left, right, _ = _overflowing_model(args)
    sh = ShardedStereo(lambda a, b: m(a, b, iters=ITERS, test_mode=True), 0, 1)
    sh.recover = False
    batch = torch.stack([left, right], 1)
    with torch.no_grad():
        sh.step(batch, (1, H, W))                 # eager warm-up (guarded: recovers, safe mode on)
        ops.set_range_safe(False)                 # capture the overflowing mode-2 graph
        ops.range_overflowed(reset=True)
        sh.capture(batch)
        ops.range_overflowed(reset=True)
        out = sh.step(batch, (1, H, W)).clone()
    torch.cuda.synchronize()
    assert bool(torch.isnan(out).all())
    with pytest.raises(ops.RangeError):
        ops.check_range()


def test_context_pre_has_no_mixed_scale_chunk(lib, monkeypatch):
    """The same scaled model with gru04.conv0's context part hoisted (update.CTX_PRE, the default): inp[0]
    is convolved alone, so no block mixes its 2^-14 chunk with the motion features -- no overflow, no
    recovery, and the oracle's result."""
    from foundationstereo_amd import update
    monkeypatch.setattr(ops, "_SPLIT_MAXPIX", 10 ** 9)
    monkeypatch.setattr(update, "CTX_PRE", True)
    args = synth.make_args(max_disp=MD, corr_levels=L, vit_size="vits")
    m, left, right, ref = _overflowing_model(args)
    ops.set_range_safe(False)
    ops.range_overflowed(reset=True)
    n0 = ops.RANGE_RECOVERIES[0]
    with torch.no_grad():
        out = m(left, right, iters=ITERS, test_mode=True)
    assert ops.RANGE_RECOVERIES[0] == n0 and not ops.range_overflowed(reset=True)
    d = float((out.cpu() - ref).abs().max())
    assert d < 1e-3, d
