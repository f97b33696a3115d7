#!/usr/bin/env python3
"""Throughput of the FoundationStereo hot path on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2] [--with-backbone]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N ...

A step = one ``FoundationStereo.forward(test_mode=True)`` over this rank's
pairs: cost-volume build, 3D filtering, context net, geometry encoding, 32
refinement iterations (lookup + ConvGRU update), convex upsampling.  Inputs
(images and the synthetic backbone's feature maps) are resident
in HBM before the timed region; the backbone is not run (``--with-backbone``: a secondary line
whose timed forward also runs the real ``Feature`` on the HIP engine).
Multi-GPU: rank 0 scatters each rank its shard of the image batch every step
and the disparities are all-gathered back (RCCL over xGMI), weights broadcast
once.

Rank 0 prints ONE JSON line.  ``roofline`` is the dominant HBM-bound kernel
(the per-iteration geometry lookup), timed with HIP events on its launch
stream over the timed region; ``cpu_baseline`` is the CPU oracle run on the
host cores for one pair of the same workload (N=1, rank 0 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from foundationstereo_amd import dist as fdist  # noqa: E402
from foundationstereo_amd import synth  # noqa: E402

HBM_PEAK = 8.0e12  # MI355X HBM3E spec, B/s (MI355X_MICROARCH.md chip table)
MFMA_F16_PEAK = 2.5e15  # dense fp16 MFMA, FLOP/s (MI355X_MICROARCH.md; no sparsity)
MFMA_F32_PEAK = 157.3e12  # f32-input MFMA (v_mfma_f32_32x32x2_f32), FLOP/s (MI355X_MICROARCH.md)
GEO_KERNELS = ("comb", "norm", "corr", "volpyr", "lookup")   # instrumented with the in-kernel clock

# BASELINE.json configs (name -> H, W, max_disp, iters, vit, pairs per GPU)
CONFIGS = {
    "cfg1": (256, 320, 64, 8, "vits", 1),     # 320x240 padded to /32
    "cfg2": (480, 640, 192, 32, "vits", 1),
    "cfg3": (480, 640, 192, 32, "vitl", 4),   # batch 32 over 8 GPUs
    "cfg4": (384, 1248, 256, 32, "vitl", 1),  # batch 8 over 8 GPUs
    "cfg5": (1024, 1536, 320, 22, "vitl", 1),  # --hiera: run_hierachical, 768x512 coarse + full pass
    "tiny": (64, 96, 32, 4, "vits", 1),
}
HIERA = {"cfg5"}


def pass_sizes(config, H, W):
    """Image sizes the forward passes of ``config`` see: the /32-padded half-size coarse pass and
    the full pass for run_hierachical (core/foundation_stereo.py:257-274), else just (H, W)."""
    if config not in HIERA:
        return [(H, W)]
    hs, ws = int(H * 0.5), int(W * 0.5)
    return [(hs + (-hs) % 32, ws + (-ws) % 32), (H + (-H) % 32, W + (-W) % 32)]


def lookup_bytes(B, H4, W4, Cv, L, r):
    """Algorithmic HBM bytes of one lookup launch: read disp, read
    the 2r+2 touched taps of Cv+1 channels per level, write 2r+1 of them."""
    K = 2 * r + 1
    N = H4 * W4
    return 4 * B * N * (1 + L * (Cv + 1) * (K + 1) + L * K * (Cv + 1))


def build_bytes(B, C, H4, W4, D4, Cs=28):
    """Algorithmic bytes of the fused comb-volume+stem kernel: read fl, fr, A, Bm; write (B,Cs,D4,H4,W4)."""
    N = H4 * W4
    return 4 * B * N * (2 * C + 2 * Cs + Cs * D4)


def allpairs_bytes(B, C, H4, W4, L):
    """All-pairs correlation pyramid: read fl, fr once, write the L levels (B,H4,W4,W4>>i)."""
    N = H4 * W4
    return 4 * B * (2 * C * N + sum(N * (W4 >> i) for i in range(L)))


def allpairs_flops(B, C, H4, W4):
    """The dense feature x feature contraction: 2*C multiply-adds per (w1, w2) pair of every row."""
    return 2 * B * C * H4 * W4 * W4


def volpyr_bytes(B, Cv, D4, H4, W4, L):
    """Filtered-volume pyramid: read level 0, write levels 1..L-1."""
    N = H4 * W4
    return 4 * B * N * Cv * (D4 + sum(D4 >> i for i in range(1, L)))


def make_model(args, device, rank):
    from foundationstereo_amd.foundation_stereo import FoundationStereo
    m = FoundationStereo(args).eval()
    if rank == 0:
        synth.init_module_(m, seed=1234)
    m = m.to(device)
    fdist.broadcast_module_(m, src=0)
    return m


def cpu_baseline(args, H, W, iters, threads, hiera=False, pair=0):
    """Time the CPU oracle on one pair of the same workload on the host cores: global pair ``pair``
    of the bench's batch (images and backbone features seeded 0x5EED + pair, as the ranks make them;
    with ``args.backbone == "real"`` the features come from the oracle's backbone restatement)."""
    import oracle
    torch.set_num_threads(threads)
    from foundationstereo_amd.foundation_stereo import FoundationStereo
    m = FoundationStereo(args)
    synth.init_module_(m, seed=1234)
    P = {k: v.float() if v.is_floating_point() else v for k, v in m.state_dict().items()}
    seed = 0x5EED + pair
    left, right = synth.stereo_images(1, H, W, seed=seed)
    T = oracle.StageTimer()
    t0 = time.perf_counter()
    with torch.no_grad():
        if args.get("backbone") == "real" and not hiera:
            from oracle import backbone_oracle
            T.mark("backbone")
            mean = torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)
            std = torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)
            ims = (torch.from_numpy(np.concatenate([left, right])) / 255.0 - mean) / std
            feats, vf = backbone_oracle.feature_forward(P, "feature.", ims, args.vit_size)
            out = oracle.oracle_forward(P, args, torch.from_numpy(left), torch.from_numpy(right),
                                        [f[:1] for f in feats], [f[1:] for f in feats], vf[:1], iters=iters, timer=T)
        elif hiera:
            def features(B, h, w):
                fl, fr, vf = synth.backbone_features(B, h, w, args.vit_size, seed=seed, shift_px=8)
                return [torch.from_numpy(a) for a in fl], [torch.from_numpy(a) for a in fr], torch.from_numpy(vf)
            out = oracle.oracle_hierarchical(P, args, torch.from_numpy(left), torch.from_numpy(right), features,
                                       iters=iters, timer=T)
        else:
            fl, fr, vf = synth.backbone_features(1, H, W, args.vit_size, seed=seed, shift_px=8)
            out = oracle.oracle_forward(P, args, torch.from_numpy(left), torch.from_numpy(right),
                                  [torch.from_numpy(a) for a in fl], [torch.from_numpy(a) for a in fr],
                                  torch.from_numpy(vf), iters=iters, timer=T)
    dt = time.perf_counter() - t0
    return dt, T.stages, out


def parity_block(out, refs, vs):
    """``parity`` of the line: max |dd| of the gathered output's pairs ``refs`` (global pair index ->
    the oracle's disparity for it) -- at N > 1 pair 0 (rank 0's) and the last pair (the last rank's,
    through the all-gather)."""
    per = {int(i): float((out[i].float().cpu() - r.float()).abs().max()) for i, r in refs.items()}
    dd = max(per.values())
    return {"max_abs_dd_px": dd, "vs": vs, "pairs_checked": sorted(per), "per_pair_dd_px": per,
            "tolerance_px": 1e-3, "ok": dd < 1e-3}


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int, argv) -> int:
    """``--gpus N`` (N > 1) without a torchrun environment: start N ranks of this script, one
    process per GPU, with torch.distributed.run on 127.0.0.1 and return their exit status.  This
    parent process never initialises the GPU (no HIP call happens before this point) and does not
    exec itself: the ranks are child processes."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__), *argv]
    print(f"[bench] launching {n} ranks: {' '.join(cmd[1:])}", file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=dict(os.environ))


def _world_info(world):
    """(world_size, backend) as torch.distributed reports them (a single process has no group)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), str(dist.get_backend())
    return world, "none (single process)"


def dist_selftest(a):
    """``--dist-selftest``: the launch / shard / gather / timing / reporting machinery of this bench
    with a stand-in per-pair function on CPU tensors over gloo -- no model, no HIP kernels (the CPU
    test of ``--gpus N``'s rank spawning, tests/test_bench_launch.py).  Its line says so in ``data``
    and is not a measurement."""
    rank, _, world = fdist.init_from_env("gloo")
    wsz, backend = _world_info(world)
    assert wsz == a.gpus, f"rank {rank}: world size {wsz} != --gpus {a.gpus}"
    B, H, W = 2 * world, 16, 24
    g = torch.Generator().manual_seed(7)
    full = torch.rand(B, 2, 3, H, W, generator=g)
    batch = full if rank == 0 else torch.zeros_like(full)
    runner = fdist.ShardedStereo(lambda lf, rt: (lf - rt).abs().mean(1, keepdim=True), rank, world)
    for _ in range(a.warmup):
        runner.step(batch, (1, H, W))
    if world > 1:
        torch.distributed.barrier()
    runner.timing = []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        out = runner.step(batch, (1, H, W))
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    attribution = fdist.rank_attribution(runner, elapsed, a.steps, torch.device("cpu"))
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    ok = bool(torch.allclose(out, (full[:, 0] - full[:, 1]).abs().mean(1, keepdim=True)))
    if rank == 0:
        ref = (full[:, 0] - full[:, 1]).abs().mean(1, keepdim=True)
        parity = parity_block(out, {0: ref[0], B - 1: ref[B - 1]} if world > 1 else {0: ref[0]},
                              "the stand-in function on the host")
        print(json.dumps({"metric": "dist self-test (no model)", "value": a.steps * B / elapsed, "unit": "pairs/s",
                          "n_gpus": wsz, "world_size": wsz, "backend": backend, "steps": a.steps,
                          "warmup": a.warmup, "gathered_ok": ok, "parity": parity, **attribution,
                          "data": "dist self-test: stand-in per-pair function on CPU tensors, not a measurement"}),
              flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()
    assert ok, "gathered batch differs from the stand-in function"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="cfg2", choices=sorted(CONFIGS))
    ap.add_argument("--corr-levels", type=int, default=4)
    ap.add_argument("--pairs-per-gpu", type=int, default=0, help="override the config's pairs per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cudnn-benchmark", type=int, default=int(os.environ.get("FSMI_CUDNN_BENCHMARK", "0")),
                    help="MIOpen Find (exhaustive, slow first call) instead of immediate-mode heuristics")
    ap.add_argument("--mixed-precision", action="store_true",
                    help="fp16 autocast for the dense convs (the reference GPU default); volumes/lookup stay fp32")
    ap.add_argument("--graph", type=int, default=1,
                    help="replay each rank's forward as one captured hipGraph (after eager warmup)")
    ap.add_argument("--conv-engine", default="fsmi", choices=["fsmi", "miopen"],
                    help="refinement-loop convs: halo-tiled split-precision MFMA kernels or MIOpen (A/B)")
    ap.add_argument("--precision", default=os.environ.get("FSMI_PRECISION", "parity"), choices=["parity", "fast"],
                    help="parity: 3 fp16 MFMA products per conv MAC (~22-bit split, the headline); fast: one "
                         "fp16 product (the reference's fp16-autocast GPU precision; |dd| reported, not parity)")
    ap.add_argument("--dist", action="store_true",
                    help="create the torch.distributed process group (RCCL) even at one rank, so the step's "
                         "scatter / all-gather run as collectives")
    ap.add_argument("--with-backbone", action="store_true",
                    help="secondary line: the timed forward also runs the real backbone (Feature: EdgeNeXt-S + "
                         "DepthAnythingV2 ViT + DPT, core/extractor.py:323-369) on the HIP engine instead of "
                         "reading preset features (the headline stays backbone-excluded, as north_star names)")
    ap.add_argument("--dist-selftest", action="store_true",
                    help="CPU/gloo self-test of the rank launch and sharding machinery (no model, not a measurement)")
    a = ap.parse_args()
    if a.gpus < 1:
        ap.error("--gpus must be >= 1")
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a.gpus, sys.argv[1:]))
    if a.dist_selftest:
        return dist_selftest(a)
    os.environ["FSMI_PRECISION"] = a.precision      # read by _lib.load(): libfsmi.so / libfsmi_fast.so
    from foundationstereo_amd import update as fupdate
    fupdate.CONV_ENGINE = a.conv_engine

    rank, local, world = fdist.init_from_env("nccl", force=a.dist)
    wsz, backend = _world_info(world)
    if wsz != a.gpus:
        raise SystemExit(f"bench.py: rank {rank} sees world size {wsz} but --gpus {a.gpus}")
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    torch.backends.cudnn.benchmark = bool(a.cudnn_benchmark)
    t_setup = time.perf_counter()
    H, W, md, iters, vit, per_gpu = CONFIGS[a.config]
    if a.pairs_per_gpu:
        per_gpu = a.pairs_per_gpu
    L = a.corr_levels
    args = synth.make_args(max_disp=md, corr_levels=L, vit_size=vit, mixed_precision=a.mixed_precision)
    if a.with_backbone:
        if a.config in HIERA:
            raise SystemExit("bench.py: --with-backbone is for the single-pass configs")
        args["backbone"] = "real"
    model = make_model(args, device, rank)

    from foundationstereo_amd import _lib, ops
    _lib.load()
    B = per_gpu * world
    lo, hi = fdist.shard_range(B, rank, world)
    # this rank's backbone output, resident in HBM (seed = 0x5EED + global pair index), per pass size
    sizes = pass_sizes(a.config, H, W)
    for (ph, pw) in ([] if a.with_backbone else sizes):
        feats = [synth.backbone_features(1, ph, pw, vit, seed=0x5EED + i, shift_px=8) for i in range(lo, hi)]
        fl = [torch.from_numpy(np.concatenate([f[0][j] for f in feats])).to(device) for j in range(4)]
        fr = [torch.from_numpy(np.concatenate([f[1][j] for f in feats])).to(device) for j in range(4)]
        vf = torch.from_numpy(np.concatenate([f[2] for f in feats])).to(device)
        model.feature.set_features(fl, fr, vf, size=(ph, pw))
    if rank == 0:
        left, right = synth.stereo_images(B, H, W)
        batch = torch.from_numpy(np.stack([left, right], 1)).to(device)
    else:   # only the shape is read on the receiving ranks: no full-batch buffer
        batch = torch.empty((1, 1, 1, 1, 1), device=device).expand(B, 2, 3, H, W)

    def fn(lft, rgt):
        if a.config in HIERA:
            return model.run_hierachical(lft, rgt, iters=iters, test_mode=True)
        return model(lft, rgt, iters=iters, test_mode=True)

    runner = fdist.ShardedStereo(fn, rank, world)
    # no host synchronisation per replay: a replay whose convs left fp16's range returns NaN (the
    # captured forward's last node, ops.range_poison_) and the flag is read once after the timed
    # region (`range_overflow`); the library default reads it per replay and recovers (1.4 % here)
    runner.recover = False

    def step():
        with torch.no_grad():
            return runner.step(batch, (1, H, W))

    t_warm = time.perf_counter()
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if rank == 0:
        print(f"[bench] setup {t_warm - t_setup:.1f}s warmup {time.perf_counter() - t_warm:.1f}s", file=sys.stderr)
    if a.graph:
        # the captured lookups carry the in-kernel clock (timer mode 2): after the timed replays their
        # stamps hold the last replay's launches, i.e. the lookup as it runs inside the timed step,
        # beside the other streams' convs (what rocprof's per-launch average of this command sees)
        step_clock = os.environ.get("FSMI_BENCH_STEP_CLOCK", "1") != "0"
        if step_clock:
            ops.timer_enable(True, in_capture=True)
        with torch.no_grad():
            runner.capture(batch)
        if step_clock:
            ops.timer_enable(False)
        step()
        torch.cuda.synchronize()
    else:
        ops.timer_enable(True)
        ops.timer_reset()
    if world > 1:
        torch.distributed.barrier()
        runner.timing = []          # per-rank scatter / forward / all-gather spans (events, no sync)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        out = step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    attribution = fdist.rank_attribution(runner, elapsed, a.steps, device) if world > 1 else {}
    runner.timing = None
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    # the timed replays' range flag, read before anything else runs: the eager timing pass below
    # goes through ops.guarded, which resets the flag.  A replay that overflowed also NaN-fills its
    # output (the captured forward's last node, ops.range_poison_); both are reported
    range_overflow = ops.range_overflowed(reset=False)
    out_finite = bool(torch.isfinite(out).all())
    # the timed step's own launches (the last replay), by the kernels' clocks baked into the graph
    in_step = {k: ops.timer_query_clock(k, captured=True) for k in GEO_KERNELS} if a.graph else {}
    lk_step_ms, lk_step_n = in_step.get("lookup", (0.0, 0))
    if a.graph:
        # graph replays carry no per-kernel events (HIP rejects external event nodes during
        # capture): time the kernels over one eager pass of the identical step instead, on one
        # stream -- with the side-stream overlap on, a kernel's event span would include the
        # time it shares the chip with another stream's kernels
        overlap, fupdate.OVERLAP = fupdate.OVERLAP, False
        ops.timer_enable(True)
        ops.timer_reset()
        runner._graph, saved = None, runner._graph
        step()
        runner._graph = saved
        fupdate.OVERLAP = overlap
    lk_ms, lk_n = ops.timer_query("lookup")
    cb_ms, cb_n = ops.timer_query("comb")
    cv_ms, cv_n = ops.timer_query("conv2d")
    # the kernels' own clocks (first block start .. last wave end, stores acknowledged): the
    # roofline duration; the event spans above also hold the event-record latency around a launch
    lk_ev_ms, cb_ev_ms = lk_ms, cb_ms
    lk_ck_ms, lk_ck_n = ops.timer_query_clock("lookup")
    cb_ck_ms, cb_ck_n = ops.timer_query_clock("comb")
    eager_clock = {k: ops.timer_query_clock(k) for k in GEO_KERNELS}
    if not a.graph:
        in_step = eager_clock
    cv_flops = ops.conv_flops()
    range_overflow_eager = ops.range_overflowed(reset=True)   # the timing pass after the timed region
    # roofline durations, each the live measurement that agrees with rocprof's per-launch average
    # (profiles/*kernel_stats.csv): a single event-bracketed launch also holds ~5 us of
    # event-record latency (`avg_us_events`, kept for reference).
    # * lookup: the kernel's own clock over the eager pass's 32 launches (first wave start to last
    #   wave end, stores acknowledged).  Replaying one launch back to back is cache-warm (its 100 MB
    #   pyramid stays in the 256 MB MALL: 35 us) and would overstate the forward's rate.
    # * build (write-dominated; the clock stops at the L2 ack of its 103 MB of stores, before the
    #   write-back): HIP events around 20 back-to-back replays of the step's launch (identical
    #   arguments, same stream, identical outputs), which amortises the event latency.
    REPS = 20
    lk_rep = lk_ck_ms / lk_ck_n if lk_ck_n == lk_n and lk_n else None
    lk_in_step = lk_step_ms / lk_step_n if lk_step_n else None   # the timed step's own lookups (ms)
    cb_rep = ops.timer_replay("comb", REPS) if cb_n else None
    ops.timer_enable(False)

    D4 = md // 4
    bl = hi - lo
    C = synth.feature_dims(vit)[0][0]
    # algorithmic bytes per launch, averaged over the passes (one size unless hierarchical)
    lk_bytes = sum(lookup_bytes(bl, ph // 4, pw // 4, 28, L, args.corr_radius) for ph, pw in sizes) / len(sizes)
    cb_bytes = build_bytes(bl, C, sizes[-1][0] // 4, sizes[-1][1] // 4, D4)   # the replayed (last) launch
    # per forward (every pass), the algorithmic bytes / flops of each geometry kernel
    fwd_bytes = {
        "comb": sum(build_bytes(bl, C, ph // 4, pw // 4, D4) for ph, pw in sizes),
        "corr": sum(allpairs_bytes(bl, C, ph // 4, pw // 4, L) for ph, pw in sizes),   # norm + corr together
        "volpyr": sum(volpyr_bytes(bl, 28, D4, ph // 4, pw // 4, L) for ph, pw in sizes),
        "lookup": iters * sum(lookup_bytes(bl, ph // 4, pw // 4, 28, L, args.corr_radius) for ph, pw in sizes),
    }
    corr_flops = sum(allpairs_flops(bl, C, ph // 4, pw // 4) for ph, pw in sizes)
    step_ms = {k: v[0] for k, v in in_step.items()}
    step_n = {k: v[1] for k, v in in_step.items()}
    geo_ms = sum(step_ms.get(k, 0.0) for k in GEO_KERNELS)
    geo_bytes = sum(fwd_bytes.values())
    geo_complete = all(step_n.get(k, 0) > 0 for k in GEO_KERNELS) and step_n.get("lookup") == iters * len(sizes)
    lk_avg = lk_rep / 1e3 if lk_rep else (lk_ms / 1e3) / max(lk_n, 1)
    lk_head_in_step = bool(lk_in_step)
    lk_head = lk_in_step / 1e3 if lk_in_step else lk_avg          # seconds per launch, headline
    cb_avg = cb_rep / 1e3 if cb_rep else (cb_ms / 1e3) / max(cb_n, 1)     # back-to-back replays (secondary)
    cb_in_step = step_ms.get("comb", 0.0) / 1e3 / step_n["comb"] if step_n.get("comb") else None
    cb_head = cb_in_step or cb_avg
    cb_head_bytes = fwd_bytes["comb"] / len(sizes) if cb_in_step else cb_bytes
    traffic = traffic_build = None
    pmc_path = os.path.join(REPO, "profiles", f"pmc_lookup_summary_{a.config}.json")
    if not os.path.exists(pmc_path):
        pmc_path = os.path.join(REPO, "profiles", "pmc_lookup_summary.json")
    if os.path.exists(pmc_path):
        with open(pmc_path) as f:
            pmc = json.load(f)
        if pmc.get("config") == a.config and pmc.get("corr_levels") == L and pmc.get("pairs_per_gpu", 1) == per_gpu:
            traffic = pmc.get("hbm_bytes_per_launch")
            traffic_build = pmc.get("build_hbm_bytes_per_launch")

    pairs = a.steps * B
    nprod = 1 if a.precision == "fast" else 3      # fp16 MFMA products per conv MAC
    res = {
        "metric": f"stereo pairs/sec ({iters} refinement iters)",
        "value": pairs / elapsed,
        "unit": "pairs/s",
        "n_gpus": world,
        "world_size": wsz,            # torch.distributed's view (1 without a process group)
        "backend": backend,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": 1e3 * elapsed / a.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        # fp32 arithmetic throughout; the convs run as 3 fp16 MFMA products per MAC on fp16 hi/lo
        # splits (~22-bit operand mantissas, fp32 accumulation), not as fp32 MFMA
        "dtype": ("fp16 convs (1 fp16 MFMA product per MAC, fp32 accumulate; fp32 volumes + lookup)"
                  if a.precision == "fast" else
                  "f32 (3xfp16 split MFMA convs; library convs fp16 under autocast)" if a.mixed_precision
                  else "f32 (3xfp16 split MFMA)"),
        "precision": a.precision,
        "data": ("synthetic (hash-PRNG images, hash-init weights incl. the backbone)" if a.with_backbone else
                 "synthetic (hash-PRNG images + synthetic backbone features, hash-init weights)"),
        "range_overflow": range_overflow,             # set during the timed replays
        "range_overflow_timing_pass": range_overflow_eager,
        "output_finite": out_finite,
        # forwards re-run in safe range mode after their range flag came back set (ops.guarded)
        "range_recoveries": ops.RANGE_RECOVERIES[0],
        # HBM high-water mark of this rank's process (caching allocator: tensors, workspaces, the captured
        # graph's private pool) -- the 288 GB budget the per-GPU batch is sized against
        "peak_mem_gb": round(torch.cuda.max_memory_allocated(device) / 1e9, 3),
        "config": {"workload": f"{a.config}: {W}x{H}{' hierarchical' if a.config in HIERA else ''}, "
                               f"max_disp {md}, {iters} iters, {vit}, "
                               f"corr_levels {L}, {per_gpu} pair(s)/GPU; forward "
                               + ("INCL. backbone (Feature on HIP; secondary line)" if a.with_backbone
                                  else "excl. backbone"),
                   "backbone": "real" if a.with_backbone else "preset features (excluded)",
                   "global_batch": B, "resolution": f"{W}x{H}", "max_disp": md, "iters": iters,
                   "corr_levels": L, "conv_engine": a.conv_engine, "hip_graph": bool(a.graph),
                   "parallelism": f"dp{world}"},
        # headline: the lookup as it runs INSIDE the timed step (its in-kernel clock, first wave start
        # to last wave end, baked into the captured graph: the last timed replay's launches, beside the
        # other streams' kernels that share the chip and its HBM); the single-stream eager pass after
        # the timed region is kept as a secondary figure
        # N > 1: each rank's own step time and its scatter / forward / all-gather split (max over ranks
        # is `ms_per_step`); the world size every rank's process group reported
        **({"rank_attribution": attribution} if attribution else {}),
        "roofline": {"kernel": "geo_lookup", "bound": "hbm",
                     "timed_over": ("the timed step (last replay's launches)" if lk_head_in_step else
                                    "single-stream eager step after the timed region" if a.graph else "timed region"),
                     "achieved": lk_bytes / lk_head / 1e9,
                     "peak": HBM_PEAK / 1e9, "unit": "GB/s", "frac": lk_bytes / lk_head / HBM_PEAK,
                     "traffic": traffic, "algorithmic_bytes": lk_bytes, "avg_us": lk_head * 1e6,
                     "timed_by": "in-kernel clock (s_memrealtime per wave) in the captured graph" if lk_head_in_step
                                 else "in-kernel clock over the eager step's launches" if lk_rep else "hip events",
                     "launches_in_step": lk_step_n,
                     "avg_us_single_stream": lk_avg * 1e6,
                     "frac_single_stream": lk_bytes / lk_avg / HBM_PEAK,
                     "avg_us_events_single_stream": lk_ev_ms * 1e3 / max(lk_n, 1), "launches_single_stream": lk_n},
        # the refinement-loop convs (halo-tiled 3 x fp16 MFMA, split-K reduce included) hold most of
        # the step time; algorithmic = fp32 conv FLOPs, peak = dense fp16 MFMA / 3 products per MAC
        "roofline_conv": {"kernel": "conv*_halo_x3 (all halo convs: loop, 3D filter, context net)", "bound": "mfma",
                          "achieved": cv_flops / (cv_ms / 1e3) / 1e12 if cv_n else None,
                          "peak": MFMA_F16_PEAK / nprod / 1e12, "unit": "TFLOP/s",
                          "frac": cv_flops / (cv_ms / 1e3) / (MFMA_F16_PEAK / nprod) if cv_n else None,
                          "algorithmic_flops": cv_flops, "total_ms": cv_ms, "launches": cv_n},
        # the same conv FLOPs over the graph-replayed step's wall time (every other kernel of the step
        # included, the 4-stream overlap on): a lower bound on the convs' in-step rate -- the
        # single-stream figure above leaves the CUs idle that low-block-count layers do not fill
        "roofline_conv_step": {"achieved": cv_flops / (elapsed / a.steps) / 1e12 if cv_n else None,
                               "peak": MFMA_F16_PEAK / nprod / 1e12, "unit": "TFLOP/s",
                               "frac": cv_flops / (elapsed / a.steps) / (MFMA_F16_PEAK / nprod) if cv_n else None,
                               "timed_over": "timed region (whole step)"},
        # the single-pass cost-volume build INSIDE the timed step (its in-kernel clock baked into the
        # graph, like the lookup's); the back-to-back replay of one launch (MALL-warm) is secondary
        "roofline_build": {"kernel": "build_stem_kernel (gwc + concat + corr_stem[0])", "bound": "hbm",
                           "achieved": cb_head_bytes / cb_head / 1e9 if cb_n else None, "peak": HBM_PEAK / 1e9,
                           "unit": "GB/s", "frac": cb_head_bytes / cb_head / HBM_PEAK if cb_n else None,
                           "traffic": traffic_build,
                           "algorithmic_bytes": cb_head_bytes, "avg_us": cb_head * 1e6,
                           "timed_over": "the timed step (last replay's launch)" if cb_in_step else "replays",
                           "timed_by": "in-kernel clock (s_memrealtime per wave) in the captured graph" if cb_in_step
                                       else f"hip events over {REPS} back-to-back replays of the step's launch",
                           "avg_us_replay": cb_avg * 1e6, "frac_replay": cb_bytes / cb_avg / HBM_PEAK if cb_n else None,
                           "avg_us_events_single_stream": cb_ev_ms * 1e3 / max(cb_n, 1),
                           "avg_us_kernel_clock_single_stream": cb_ck_ms * 1e3 / max(cb_ck_n, 1), "launches": cb_n},
        # north star: build + correlation lookup as ONE per-pair figure -- every geometry kernel of the
        # timed step (build, all-pairs normalisation + MFMA pass, volume pyramid, the `iters` lookups)
        # by its in-step clock, against their algorithmic bytes (5.78 GB per cfg2 pair, L=4)
        "roofline_build_lookup": {
            "kernels": "build_stem + normalize_cols + allpairs_corr + volume_pyramid + geo_lookup x iters",
            "bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK / 1e9,
            "achieved": geo_bytes / (geo_ms / 1e3) / 1e9 if geo_complete else None,
            "frac": geo_bytes / (geo_ms / 1e3) / HBM_PEAK if geo_complete else None,
            "algorithmic_bytes_per_pair": geo_bytes / bl, "us_per_pair": geo_ms * 1e3 / bl,
            "timed_over": "the timed step (last replay)" if a.graph else "eager step",
            "per_kernel_us": {k: round(step_ms.get(k, 0.0) * 1e3, 2) for k in GEO_KERNELS},
            "per_kernel_launches": step_n,
            "per_kernel_bytes": fwd_bytes},
        # the one dense contraction north_star puts on MFMA: the all-pairs correlation (fp32 MFMA)
        "allpairs_mfma": {"kernel": "allpairs_corr_direct_kernel (v_mfma_f32_32x32x2_f32)", "bound": "mfma",
                          "flops": corr_flops, "unit": "TFLOP/s", "peak": MFMA_F32_PEAK / 1e12,
                          "avg_us": step_ms.get("corr", 0.0) * 1e3 / max(step_n.get("corr", 0), 1),
                          "achieved": (corr_flops / (step_ms["corr"] / 1e3) / 1e12) if step_n.get("corr") else None,
                          "frac": (corr_flops / (step_ms["corr"] / 1e3) / MFMA_F32_PEAK) if step_n.get("corr") else None,
                          "normalize_us": step_ms.get("norm", 0.0) * 1e3 / max(step_n.get("norm", 0), 1),
                          "timed_over": "the timed step (last replay)" if a.graph else "eager step"},
    }
    if rank == 0 and (world > 1 or not a.no_cpu_baseline):
        # the host cores this process is given: OMP_NUM_THREADS (16 on the GPU box = its CPU share
        # per GPU; os.cpu_count() there reports the whole machine, shared with other jobs)
        threads = int(os.environ.get("OMP_NUM_THREADS", 0)) or (os.cpu_count() or 1)
        dt, stages, ref = cpu_baseline(args, H, W, iters, threads, hiera=a.config in HIERA)
        # the oracle ran pair 0 of this very workload (same seeds): the step's own disparity vs it; at
        # N > 1 also the batch's last pair, computed by the last rank and returned by the all-gather
        # (a multi-GPU line always carries parity; --no-cpu-baseline skips it at N = 1 only)
        refs = {0: ref[0]}
        if world > 1 and B > 1:
            refs[B - 1] = cpu_baseline(args, H, W, iters, threads, hiera=a.config in HIERA, pair=B - 1)[2][0]
        res["parity"] = parity_block(out, refs, "CPU oracle (fp32), the timed step's gathered output")
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        res["cpu_baseline"] = {"value": 1.0 / dt, "unit": "pairs/s", "cores": threads, "kind": "port",
                               "cpu_model": _cpu_model(), "host_cpus": os.cpu_count(),
                               "sample": f"1 pair of {a.config} (all {iters} iterations) through the fp32 "
                                         f"torch-CPU oracle, {dt:.1f} s",
                               "stages_s": {k: round(v, 3) for k, v in stages.items()}}
    if rank == 0:
        # a multi-GPU line never prints without parity (its pairs came back through the all-gather)
        assert world == 1 or "max_abs_dd_px" in res.get("parity", {}), "multi-GPU line without parity"
        print(json.dumps(res), flush=True)
    if not out_finite:
        raise SystemExit("bench.py: the timed step returned non-finite disparities (range overflow)")
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
