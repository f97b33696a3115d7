#!/usr/bin/env python3
"""Measure the best tile config / split-K factor of every halo-conv shape the given workloads use
and MERGE them into tuning/fsmi_conv.json (read by ops.conv2d / conv2d_gate / conv3d when the
caller leaves cfg / nsplit on auto).  Run on the GPU box:

    python tools/tune_conv.py [--config cfg2 cfg3 ...] [--reps 5] [--only-cfgs 19 20 21 23]
    python tools/tune_conv.py --with-backbone --new-only     # the backbone's (Feature) conv shapes

Candidates per shape: the plain tiles (0-9 as they apply), the K-group variants (16 + 3/4/5/7:
two wave groups per block on alternate chunks, summed in LDS), for 2D 1x1 layers the pointwise
LDS-DMA tiles (24-26, conv_pw.hip), for 2D maps the pipelined-staging register tiles (32 + 2..9)
and for (17, 1, 1) volume convs the depth-blocked tile (30, conv_depth.hip), each with split-K
factors.  With
--only-cfgs only those are timed against the shape's current table entry, the better one kept.
Shapes of other workloads already in the table are kept as they are.
"""
import argparse
import json
import os
import re
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from foundationstereo_amd import ops, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", nargs="+", default=["cfg2"])
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--only-cfgs", type=int, nargs="*", default=None,
                help="time only these cfgs (plus the current table entry); keep the better")
ap.add_argument("--max-split", type=int, default=8, help="largest split-K factor to time")
ap.add_argument("--match", default="", help="only re-tune shape keys matching this regex (e.g. '_d(?!1_)' volumes)")
ap.add_argument("--with-backbone", action="store_true",
                help="record the shapes of a forward WITH the HIP backbone (Feature), not preset features")
ap.add_argument("--new-only", action="store_true", help="tune only shape keys the table does not hold yet")
ap.add_argument("--out", default=os.path.join(REPO, "tuning", "fsmi_conv.json"))
ap.add_argument("--base", default=os.path.join(REPO, "tuning", "fsmi_conv.json"),
                help="table to start from (merged into --out)")
a = ap.parse_args()
dev = torch.device("cuda:0")

import bench  # noqa: E402  (workload table)


def record_shapes(config):
    """Conv shape keys of one (2-iteration) pass of ``config``, tuning table off (all on auto)."""
    H, W, md, iters, vit, per_gpu = bench.CONFIGS[config]
    args = synth.make_args(max_disp=md, corr_levels=4, vit_size=vit)
    if a.with_backbone:
        args["backbone"] = "real"
    model = bench.make_model(args, dev, 0)
    for (ph, pw) in ([] if a.with_backbone else bench.pass_sizes(config, H, W)):
        feats = [synth.backbone_features(1, ph, pw, vit, seed=0x5EED + i, shift_px=8) for i in range(per_gpu)]
        fl = [torch.from_numpy(np.concatenate([f[0][j] for f in feats])).to(dev) for j in range(4)]
        fr = [torch.from_numpy(np.concatenate([f[1][j] for f in feats])).to(dev) for j in range(4)]
        vf = torch.from_numpy(np.concatenate([f[2] for f in feats])).to(dev)
        model.feature.set_features(fl, fr, vf, size=(ph, pw))
    left, right = synth.stereo_images(per_gpu, H, W)
    os.environ["FSMI_TUNE_DB"] = "0"
    ops._RECORD = set()
    with torch.no_grad():
        lt, rt = torch.from_numpy(left).to(dev), torch.from_numpy(right).to(dev)
        if config in bench.HIERA:
            model.run_hierachical(lt, rt, iters=2, test_mode=True)
        else:
            model(lt, rt, iters=2, test_mode=True)
    torch.cuda.synchronize()
    keys = sorted(ops._RECORD)
    ops._RECORD = None
    os.environ.pop("FSMI_TUNE_DB")
    del model
    torch.cuda.empty_cache()
    return keys


def timeit(fn):
    """GPU time per call: reps calls captured into one hipGraph and replayed (as bench.py runs the
    forward), so small layers are not timed at the host's launch rate (~17 us per eager call)."""
    fn()
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(a.reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    del g
    return e0.elapsed_time(e1) * 1e3 / (3 * a.reps)


table = {}
if os.path.exists(a.base):
    with open(a.base) as f:
        table = json.load(f)
entries = dict(table.get("entries", {}))
prev = dict(entries)
keys = sorted({k for c in a.config for k in record_shapes(c)})
if a.match:
    keys = [k for k in keys if re.search(a.match, k)]
if a.new_only:
    keys = [k for k in keys if k not in entries]
print(f"[tune] {len(keys)} conv shapes for {a.config}", file=sys.stderr)
t_start = time.time()
with torch.no_grad():
    for key in keys:
        if "s2" in key:                              # stride-2 tiles: their own table entries (s2_bench)
            continue
        ks, kd, cin, cout, B, D, Hh, Ww = (int(v) for v in re.findall(r"\d+", key))
        if kd == 1 and D == 1:
            x = torch.randn(B, cin, Hh, Ww, device=dev)
            w = torch.randn(cout, cin, ks, ks, device=dev) * 0.05
        else:
            x = torch.randn(B, cin, D, Hh, Ww, device=dev)
            w = torch.randn(cout, cin, kd, ks, ks, device=dev) * 0.05
        b = torch.randn(cout, device=dev)
        pk = ops.PackedConv(w, mode="halo")

        def run(cfg, ns):
            if x.dim() == 4:
                return ops.conv2d([x], pk, bias=b, act="relu", cfg=cfg, nsplit=ns)
            return ops.conv3d(x, pk, bias=b, act="relu", cfg=cfg, nsplit=ns)

        nck = kd * ((cin + 31) // 32)
        cfgs = ([2, 3, 4, 5] + ([0, 1] if x.dim() == 4 else []) + ([6, 7] if cout <= 64 else [])
                + ([8] if cout > 64 else []) + ([9] if cout > 128 else [])
                + ([11] if cout > 128 and x.dim() == 4 else [])
                + [16 + c for c in (3, 4, 5) + ((7,) if cout <= 64 else ()) if nck >= 2]
                + ([24, 25, 26, 27, 28, 29] if ks == 1 and x.dim() == 4 and (Hh * Ww) % 4 == 0 else []))
        if x.dim() == 4:                            # pipelined-staging variants of the register tiles
            cfgs += [32 + c for c in cfgs if 2 <= c <= 9 or c == 11]
        if x.dim() == 5 and ks == 1 and kd == 17:   # depth-blocked (17, 1, 1) tile (no split-K)
            cfgs.append(30)
        splits = [s for s in (1, 2, 3, 4, 6, 8) if s <= max(1, nck) and s <= a.max_split]
        auto = timeit(lambda: run(-1, -1))
        best = (auto, -1, -1)
        if a.only_cfgs is not None:
            cfgs = [c for c in cfgs if c in a.only_cfgs]
            old = prev.get(key)
            if old is not None:
                best = (timeit(lambda: run(old["cfg"], old["nsplit"])), old["cfg"], old["nsplit"])
        for c in cfgs:
            for s in splits:
                if 16 <= c < 24 and 2 * s > nck:   # K groups need >= 2 chunks per block
                    continue
                if c == 30 and s > 1:
                    continue
                t = timeit(lambda: run(c, s))
                if t < best[0]:
                    best = (t, c, s)
        if best[1] >= 0:
            entries[key] = {"cfg": best[1], "nsplit": best[2], "us": round(best[0], 1), "auto_us": round(auto, 1)}
        print(json.dumps({"key": key, "auto_us": round(auto, 1), "best_us": round(best[0], 1), "cfg": best[1],
                          "nsplit": best[2]}), flush=True)

os.makedirs(os.path.dirname(a.out), exist_ok=True)
configs = sorted(set(str(table.get("config", "")).split(",")) - {""} | set(a.config))
with open(a.out, "w") as f:
    json.dump({"device": torch.cuda.get_device_name(0), "config": ",".join(configs),
               "source": "tools/tune_conv.py (merged per workload)", "entries": entries}, f, indent=1, sort_keys=True)
print(f"[tune] {len(entries)} entries in {a.out} after {time.time() - t_start:.0f}s", file=sys.stderr)
