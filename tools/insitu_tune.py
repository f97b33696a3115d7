#!/usr/bin/env python3
"""In-situ conv tuning: greedy search over the tuning table with the captured end-to-end step as the
objective.  tools/tune_conv.py times every layer alone on an idle chip; inside the 4-stream
pipelined loop other streams' kernels share the CUs, so the per-layer optimum is not the
end-to-end one (e.g. the split-K cap, ops._SPLIT_CAP).  Here:

  1. one eager forward records every conv shape and its call count;
  2. per shape the (cfg, nsplit <= --max-split) candidates are timed alone (graph-timed, like
     tune_conv.py) and the 3 fastest kept;
  3. shapes in order of their share of the step (calls x table time), each alternative is put in
     the table, the forward re-captured as a hipGraph and replayed; kept if the step gets faster
     by more than --min-gain.

    python tools/insitu_tune.py [--config cfg2] [--top 30] [--write]      (GPU box)
"""
import argparse
import gc
import json
import os
import re
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from foundationstereo_amd import dist as fdist, ops, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="cfg2")
ap.add_argument("--top", type=int, default=30, help="shapes to search, by share of the step")
ap.add_argument("--alts", type=int, default=3, help="alternatives per shape")
ap.add_argument("--reps", type=int, default=12, help="graph replays per evaluation")
ap.add_argument("--min-gain", type=float, default=0.003, help="relative step gain to keep a change")
ap.add_argument("--max-split", type=int, default=4, help="largest split-K factor among the alternatives")
ap.add_argument("--write", action="store_true", help="merge the result into tuning/fsmi_conv.json")
ap.add_argument("--out", default="", help="also write the merged table here (e.g. under gpurun_out/)")
ap.add_argument("--nosplit", action="store_true", help="also try each shape's current tile without split-K")
ap.add_argument("--alts-only", action="store_true", help="skip the isolated candidate search (with --nosplit)")
ap.add_argument("--match", default="", help="regex: only shapes whose key matches")
ap.add_argument("--prefer-nosplit", type=float, default=-1.0,
                help="accept an alternative with a smaller split-K factor unless it is slower by more than this "
                     "relative amount (e.g. 0.002): fewer split-K reduce passes at equal step time")
ap.add_argument("--try", dest="try_", nargs="*", default=[],
                help="cfg:nsplit pairs tried in situ on every searched shape they are legal for (e.g. 43:1 43:2)")
a = ap.parse_args()
dev = torch.device("cuda:0")
t_start = time.time()

H, W, md, iters, vit, per_gpu = bench.CONFIGS[a.config]
args = synth.make_args(max_disp=md, corr_levels=4, vit_size=vit)
model = bench.make_model(args, dev, 0)
for (ph, pw) in bench.pass_sizes(a.config, H, W):
    feats = [synth.backbone_features(1, ph, pw, vit, seed=0x5EED + i, shift_px=8) for i in range(per_gpu)]
    fl = [torch.from_numpy(np.concatenate([f[0][j] for f in feats])).to(dev) for j in range(4)]
    fr = [torch.from_numpy(np.concatenate([f[1][j] for f in feats])).to(dev) for j in range(4)]
    vf = torch.from_numpy(np.concatenate([f[2] for f in feats])).to(dev)
    model.feature.set_features(fl, fr, vf, size=(ph, pw))
left, right = synth.stereo_images(per_gpu, H, W)
batch = torch.from_numpy(np.stack([left, right], 1)).to(dev)


def fn(lft, rgt):
    if a.config in bench.HIERA:
        return model.run_hierachical(lft, rgt, iters=iters, test_mode=True)
    return model(lft, rgt, iters=iters, test_mode=True)


runner = fdist.ShardedStereo(fn, 0, 1)
cap = a.max_split               # in-situ entries bypass ops._SPLIT_CAP (they are marked "insitu")

# 1. census (eager) + warmup
ops._TUNE = None
ops._tuned(1, 1, 1, 1, 1, 1, 1, 1, -1, -1)          # loads the table into ops._TUNE
table = ops._TUNE
ops._RECORD = {}
with torch.no_grad():
    runner.step(batch, (1, H, W))
torch.cuda.synchronize()
counts, ops._RECORD = ops._RECORD, None
with torch.no_grad():
    runner.step(batch, (1, H, W))
torch.cuda.synchronize()


def evaluate():
    """ms per step: the forward re-captured with the current table, replayed a.reps times."""
    runner._graph = None
    gc.collect()
    torch.cuda.empty_cache()
    with torch.no_grad():
        runner.capture(batch)
        for _ in range(2):
            runner._run(runner._local)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        runner._run(runner._local)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / a.reps


def graph_time(f, reps=10):
    f()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            f()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    del g
    return e0.elapsed_time(e1) * 1e3 / reps


def candidates(key):
    """the a.alts fastest (cfg, nsplit) of a shape timed alone (graph-timed), nsplit <= cap"""
    if a.alts_only:
        return [], table_us(key)
    ks, kd, cin, cout, B, D, Hh, Ww = (int(v) for v in re.findall(r"\d+", key))
    with torch.no_grad():
        if kd == 1 and D == 1:
            x = torch.randn(B, cin, Hh, Ww, device=dev)
            w = torch.randn(cout, cin, ks, ks, device=dev) * 0.05
        else:
            x = torch.randn(B, cin, D, Hh, Ww, device=dev)
            w = torch.randn(cout, cin, kd, ks, ks, device=dev) * 0.05
        b = torch.randn(cout, device=dev)
        pk = ops.PackedConv(w, mode="halo")
        nck = kd * ((cin + 31) // 32)
        cfgs = ([2, 3, 4, 5] + ([0, 1] if x.dim() == 4 else []) + ([6, 7] if cout <= 64 else [])
                + ([8] if cout > 64 else []) + ([9] if cout > 128 else [])
                + ([11] if cout > 128 and x.dim() == 4 else [])
                + [16 + c for c in (3, 4, 5) + ((7,) if cout <= 64 else ()) if nck >= 2]
                + ([24, 25, 26, 27, 28, 29] if ks == 1 and x.dim() == 4 and (Hh * Ww) % 4 == 0 else []))
        if x.dim() == 4:                            # pipelined-staging variants of the register tiles
            cfgs += [32 + c for c in cfgs if 2 <= c <= 9 or c == 11]
        if x.dim() == 5 and ks == 1 and kd == 17:   # depth-blocked (17, 1, 1) tile
            cfgs.append(30)
        res = []
        for c in cfgs:
            for s in (1, 2, 3, 4):
                if s > cap or (s > 1 and s > nck) or (c >= 16 and c < 24 and 2 * s > nck) or (c == 30 and s > 1):
                    continue
                if x.dim() == 4:
                    f = lambda: ops.conv2d([x], pk, bias=b, act="relu", cfg=c, nsplit=s)  # noqa: E731
                else:
                    f = lambda: ops.conv3d(x, pk, bias=b, act="relu", cfg=c, nsplit=s)  # noqa: E731
                res.append((graph_time(f), c, s))
    res.sort()
    return [(c, s) for _, c, s in res[:a.alts]], res[0][0]


def table_us(key):
    e = table.get(key)
    return e.get("us", 0.0) if e else 0.0


order = sorted((k for k in counts if "s2" not in k and re.search(a.match, k)),   # stride-2: s2_bench entries
               key=lambda k: -counts[k] * max(table_us(k), 1.0))[:a.top]


def legal(key, c, s):
    ks, kd, cin, cout, B, D, Hh, Ww = (int(v) for v in re.findall(r"\d+", key))
    two_d = kd == 1 and D == 1
    nck = kd * ((cin + 31) // 32)
    if s > nck:
        return False
    if c in (11, 43) or c >= 32:
        return two_d
    if 24 <= c <= 29:
        return two_d and ks == 1 and (Hh * Ww) % 4 == 0
    if c == 30:
        return not two_d and ks == 1 and kd == 17 and s == 1
    if 16 <= c < 24:
        return 2 * s <= nck
    return True
print(f"[insitu] {len(counts)} conv shapes, searching {len(order)}", file=sys.stderr, flush=True)
base = min(evaluate(), evaluate())
start = base
print(json.dumps({"start_ms": round(base, 3)}), flush=True)
changes = {}
for n, key in enumerate(order):
    cur = table.get(key)
    alts, best_alone = candidates(key)
    if a.nosplit and cur is not None and (cur["cfg"], 1) not in alts and cur["cfg"] != 30:
        alts = [(cur["cfg"], 1)] + alts          # no split-K: other streams fill the tail in situ
    for pair in a.try_:
        c, s = (int(v) for v in pair.split(":"))
        if (c, s) not in alts and legal(key, c, s):
            alts.append((c, s))
    print(f"[insitu] {n + 1}/{len(order)} {key} x{counts[key]}: alternatives {alts}, step {base:.3f} ms "
          f"({(time.time() - t_start) / 60:.1f} min)", file=sys.stderr, flush=True)
    for (c, s) in alts:
        if cur is not None:
            eff = cur["nsplit"] if cur.get("insitu") or not ops._SPLIT_CAP else min(cur["nsplit"], ops._SPLIT_CAP)
            if cur["cfg"] == c and eff == s:
                continue
        table[key] = {"cfg": c, "nsplit": s, "us": round(best_alone, 1), "insitu": True}
        t = min(evaluate(), evaluate())
        cur_split = cur["nsplit"] if cur is not None else 1
        fewer = a.prefer_nosplit >= 0 and s < cur_split and t < base * (1 + a.prefer_nosplit)
        if t < base * (1 - a.min_gain) or fewer:
            print(json.dumps({"key": key, "cfg": c, "nsplit": s, "ms": round(t, 3), "was_ms": round(base, 3)}),
                  flush=True)
            base, cur = t, table[key]
            changes[key] = cur
        elif cur is not None:
            table[key] = cur
        else:
            del table[key]
    base = min(base, evaluate())
final = min(evaluate(), evaluate())
print(json.dumps({"start_ms": round(start, 3), "final_ms": round(final, 3), "changes": len(changes),
                  "minutes": round((time.time() - t_start) / 60, 1)}), flush=True)
if a.write and changes and final < start:
    with open(ops._TUNE_PATH) as f:
        db = json.load(f)
    db["entries"].update(changes)
    db["source"] = "tools/tune_conv.py (merged per workload) + tools/insitu_tune.py (end-to-end greedy)"
    with open(ops._TUNE_PATH, "w") as f:
        json.dump(db, f, indent=1, sort_keys=True)
    print(f"[insitu] wrote {len(changes)} changes to {ops._TUNE_PATH}", file=sys.stderr)
if a.out and changes and final < start:
    with open(ops._TUNE_PATH) as f:
        db = json.load(f)
    db["entries"].update(changes)
    with open(a.out, "w") as f:
        json.dump(db, f, indent=1, sort_keys=True)
