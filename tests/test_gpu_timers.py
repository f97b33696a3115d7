"""The measurement hooks bench.py reads (include/fsmi.h fsmi_timer_*): the in-kernel lookup clock,
eagerly and -- timer mode 2 -- baked into a captured hipGraph, whose replays rewrite the stamps
(bench.py's in-step roofline)."""
import pytest
import torch

from foundationstereo_amd import synth


@pytest.mark.gpu
def test_lookup_clock_in_captured_graph():
    from foundationstereo_amd import ops
    dev = torch.device("cuda:0")
    B, Cv, D, H, W, L = 1, 28, 48, 24, 64, 4
    vol = torch.from_numpy(synth.normal(81, (B, Cv, D, H, W))).to(dev)
    f1, f2 = (torch.from_numpy(synth.normal(s, (B, 64, H, W))).to(dev) for s in (82, 83))
    corr = ops.allpairs_corr(f1, f2, L)
    pyr = ops.volume_pyramid(vol, L)
    disp = torch.from_numpy(synth.uniform(84, (B, 1, H, W), 0.0, D - 1.0)).to(dev)
    ref = ops.geo_lookup(pyr, corr, disp, 4)
    torch.cuda.synchronize()
    try:
        ops.timer_enable(True, in_capture=True)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = ops.geo_lookup(pyr, corr, disp, 4)
            out2 = ops.geo_lookup(pyr, corr, disp, 4)
            corr_g = ops.allpairs_corr(f1, f2, L)
            pyr_g = ops.volume_pyramid(vol, L)
        ops.timer_enable(False)
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        ms, n = ops.timer_query_clock("lookup", captured=True)
        assert n == 2 and 0.0 < ms / n < 5.0, (ms, n)       # both captured launches stamped, sane us
        assert ops.timer_query_clock("lookup")[1] == 0       # no eager launch since the enable
        for k in ("corr", "norm", "volpyr"):                 # the other geometry kernels' in-step clocks
            ms, n = ops.timer_query_clock(k, captured=True)
            assert n == 1 and 0.0 < ms < 5.0, (k, ms, n)
        assert torch.equal(out, ref) and torch.equal(out2, ref)
        for a_, b_ in zip(corr_g + pyr_g[1:], corr + pyr[1:]):
            assert torch.equal(a_, b_)
        # mode 1: captured launches carry no clock; the records of the mode-2 graph survive the
        # new session (its replays keep writing those slots), until released
        ops.timer_enable(True)
        g2 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g2):
            ops.geo_lookup(pyr, corr, disp, 4)
        g2.replay()
        ops.geo_lookup(pyr, corr, disp, 4)                   # one eager launch: clocked in mode 1
        torch.cuda.synchronize()
        assert ops.timer_query_clock("lookup")[1] == 1
        assert ops.timer_query_clock("lookup", captured=True)[1] == 2
        g.replay()
        torch.cuda.synchronize()
        assert ops.timer_query_clock("lookup", captured=True)[1] == 2
        del g
        ops.timer_release_captured()
        assert ops.timer_query_clock("lookup", captured=True)[1] == 0
        # release starts a clean session (timing still on): the eager records are gone, and a new eager
        # launch gets a zeroed slot -- a sane duration, not another launch's stale stamps
        assert ops.timer_query_clock("lookup")[1] == 0
        ops.geo_lookup(pyr, corr, disp, 4)
        torch.cuda.synchronize()
        ms, n = ops.timer_query_clock("lookup")
        assert n == 1 and 0.0 < ms < 5.0, (ms, n)
    finally:
        ops.timer_enable(False)


@pytest.mark.gpu
def test_clock_arena_holds_a_cfg5_step():
    """bench.py's timer mode 2 at cfg5 scale: 32 lookups of the 1536x1024 pass (384 x 256 at 1/4, 49k waves
    each) baked into a graph, then 32 eager ones -- ~6M stamps, beyond the 4M arena that failed the cfg3 /
    cfg5 bench lines; every launch must be recorded (a full arena makes the query raise)."""
    from foundationstereo_amd import ops
    dev = torch.device("cuda:0")
    B, Cv, D, H, W, L = 1, 28, 48, 256, 384, 4
    vol = torch.from_numpy(synth.normal(91, (B, Cv, D, H, W))).to(dev)
    f1, f2 = (torch.from_numpy(synth.normal(s, (B, 32, H, W))).to(dev) for s in (92, 93))
    corr = ops.allpairs_corr(f1, f2, L)
    pyr = ops.volume_pyramid(vol, L)
    disp = torch.from_numpy(synth.uniform(94, (B, 1, H, W), 0.0, D - 1.0)).to(dev)
    torch.cuda.synchronize()
    try:
        ops.timer_enable(True, in_capture=True)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(32):
                ops.geo_lookup(pyr, corr, disp, 4)
        g.replay()
        for _ in range(32):
            ops.geo_lookup(pyr, corr, disp, 4)
        torch.cuda.synchronize()
        assert ops.timer_query_clock("lookup", captured=True)[1] == 32
        assert ops.timer_query_clock("lookup")[1] == 32
        del g
        ops.timer_release_captured()
    finally:
        ops.timer_enable(False)
