#!/usr/bin/env python3
"""Timeline of the graph-replayed forward WITHOUT a profiler: every instrumented kernel of the captured
forward stamps its first wave start and last wave end (s_memrealtime, 10 ns) into a slot baked into the
graph (timer mode 3, include/fsmi.h fsmi_timer_dump_captured; the timeline build _lib/libfsmi_timeline.so,
whose kernels carry the stamps -- the product build compiles them out); after the replays the last replay's
stamps are read back.  rocprofv3's kernel trace re-maps the graph onto its own hardware queues and
slows the step (~17 vs ~21 pairs/s at cfg2), so its per-iteration picture is not the timed step's.

    python tools/replay_timeline.py [--config cfg2] [--iter 16] [--out gpurun_out/r5/replay_timeline.txt]

Prints, for iteration ``--iter`` (lookup(t) start .. lookup(t+1) start): every stamped launch with its
capture stream (main / motion / branch / pipeline), start / end in us from lookup(t), duration and tag;
the busy time per stream; and the chain that sets the iteration's length, walked back from lookup(t+1)
through the captured graph's dependencies: each launch's own-stream predecessor plus, for every
cross-stream wait its stream issued (logged with its capture position, update.WAIT_LOG), the waited
stream's last launch before the wait; each step takes the dependency that finished last.  (Round 5's
tool took the latest-ending launch of ANY stream at each step, which walked into the pipeline stream
whenever one of its convs happened to end just before a main-stream launch.)  Kernels without a clock (the
few non-fsmi ops, MIOpen) are absent, so gaps in the chain can hide them.  Also the whole step: span,
kernel time per stream and the sum over launches per tag family.
"""
import argparse
import json
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
# the conv / MLP / aux kernels carry clocks only in the timeline build (python -c "from
# foundationstereo_amd import build; build.build_timeline()")
os.environ.setdefault("FSMI_LIB", os.path.join(REPO, "foundationstereo_amd", "_lib", "libfsmi_timeline.so"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from foundationstereo_amd import _lib, ops, synth  # noqa: E402
from foundationstereo_amd import update as fupdate  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="cfg2")
ap.add_argument("--iter", type=int, default=16)
ap.add_argument("--replays", type=int, default=5)
ap.add_argument("--out", default="")
ap.add_argument("--list", default="", help="regex: also list every launch of the step whose tag matches")
a = ap.parse_args()
dev = torch.device("cuda:0")
H, W, md, iters, vit, per = bench.CONFIGS[a.config]
args = synth.make_args(max_disp=md, corr_levels=4, vit_size=vit)
model = bench.make_model(args, dev, 0)
feats = [synth.backbone_features(1, H, W, vit, seed=0x5EED + i, shift_px=8) for i in range(per)]
fl = [torch.from_numpy(np.concatenate([f[0][j] for f in feats])).to(dev) for j in range(4)]
fr = [torch.from_numpy(np.concatenate([f[1][j] for f in feats])).to(dev) for j in range(4)]
vf = torch.from_numpy(np.concatenate([f[2] for f in feats])).to(dev)
model.feature.set_features(fl, fr, vf, size=(H, W))
left, right = synth.stereo_images(per, H, W)
L, R = torch.from_numpy(left).to(dev), torch.from_numpy(right).to(dev)
lib = _lib.load()
with torch.no_grad():
    for _ in range(2):
        model(L, R, iters=iters, test_mode=True)
    torch.cuda.synchronize()
    ops.timer_enable(True, timeline=True)
    fupdate.WAIT_LOG = []                    # the capture's cross-stream waits, by capture position
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        model(L, R, iters=iters, test_mode=True)
    waits, fupdate.WAIT_LOG = fupdate.WAIT_LOG, None
    ops.timer_enable(False)
for _ in range(a.replays):
    g.replay()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
g.replay()
e1.record()
torch.cuda.synchronize()
step_ms = e0.elapsed_time(e1)
names = {}
for idx, nm in ((0, "motion"), (1, "branch"), (3, "pipeline")):
    names[fupdate._side_stream(dev, idx).cuda_stream] = nm
recs = [{"k": k, "sp": sp, "stream": names.get(sp, "main"), "s": t0, "e": t1, "tag": tag or _lib.KERNELS[k], "i": i}
        for i, (k, sp, t0, t1, tag) in enumerate(ops.timer_dump_captured())]
# the captured graph's dependencies of each launch (capture position i): its stream's previous launch,
# and for every wait its stream issued since that launch (capture position <= i), the waited stream's
# last launch captured before the wait
by_pos = list(recs)
last_on = {}
deps = {}
for r in by_pos:
    prev = last_on.get(r["sp"])
    d = [prev] if prev is not None else []
    lo = prev["i"] if prev is not None else -1
    for (ws, wd, k) in waits:
        if ws == r["sp"] and lo < k <= r["i"]:
            cand = [q for q in by_pos[:k] if q["sp"] == wd]
            if cand:
                d.append(cand[-1])
    deps[r["i"]] = d
    last_on[r["sp"]] = r
recs = [r for r in recs if r["s"] and r["e"] >= r["s"]]
recs.sort(key=lambda r: r["s"])
out = []


def emit(x=""):
    out.append(x)
    print(x)


t_first, t_last = recs[0]["s"], max(r["e"] for r in recs)
emit(f"{a.config}: replay device time {step_ms:.2f} ms (events); stamped span {(t_last - t_first) / 1e5:.2f} ms, "
     f"{len(recs)} stamped launches")
per_stream = {}
for r in recs:
    per_stream[r["stream"]] = per_stream.get(r["stream"], 0) + r["e"] - r["s"]
emit("kernel time per stream (whole step): " + ", ".join(f"{k} {v / 1e5:.2f} ms" for k, v in sorted(per_stream.items())))
fam = {}
for r in recs:
    f = re.sub(r" (ci|co|d|h|w|ns)\d+", "", r["tag"])
    fam[f] = fam.get(f, 0) + r["e"] - r["s"]
emit("top launch families (summed kernel time, ms): " + json.dumps(
    {k: round(v / 1e5, 2) for k, v in sorted(fam.items(), key=lambda x: -x[1])[:12]}))
lk = [i for i, r in enumerate(recs) if r["k"] == _lib.KERNELS.index("lookup")]
if lk:
    # before the refinement loop: context net, volume build, 3D filtering, geometry pyramids
    t_l0 = recs[lk[0]]["s"]
    pre = [r for r in recs if r["s"] < t_l0]
    fam_pre = {}
    for r in pre:
        f = re.sub(r" (ci|co|h|w|ns)\d+", "", r["tag"])
        fam_pre[f] = fam_pre.get(f, 0) + min(r["e"], t_l0) - r["s"]
    emit(f"pre-loop: {(t_l0 - t_first) / 1e5:.2f} ms from the first stamped launch to lookup 0, {len(pre)} launches; "
         f"post-loop: {(t_last - recs[lk[-1]]['e']) / 1e5:.2f} ms after the last lookup")
    emit("  pre-loop kernel time by family (ms): " + json.dumps(
        {k: round(v / 1e5, 3) for k, v in sorted(fam_pre.items(), key=lambda x: -x[1])[:16]}))
    # the last iteration (from its lookup) and the post-loop tail (mask head, spx upsampling), every launch
    t_ll = recs[lk[-1]]["s"]
    emit("  last iteration + post-loop launches (stream, start / end us from the last lookup, us, tag):")
    for r in [r for r in recs if r["e"] > t_ll]:
        emit(f"  {r['stream']:>8} {(r['s'] - t_ll) / 100:8.1f} {(r['e'] - t_ll) / 100:8.1f} {(r['e'] - r['s']) / 100:7.1f}  {r['tag']}")
if len(lk) > a.iter + 1:
    first, nxt = recs[lk[a.iter]], recs[lk[a.iter + 1]]
    t0, t1 = first["s"], nxt["s"]
    sel = [r for r in recs if r["e"] > t0 and r["s"] < t1]
    emit(f"iteration {a.iter}: {(t1 - t0) / 100:.1f} us lookup to lookup, {len(sel)} stamped launches")
    for r in sel:
        emit(f"  {r['stream']:>8} {(r['s'] - t0) / 100:8.1f} {(r['e'] - t0) / 100:8.1f} {(r['e'] - r['s']) / 100:7.1f}  {r['tag']}")
    busy = {}
    for r in sel:
        busy[r["stream"]] = busy.get(r["stream"], 0) + min(r["e"], t1) - max(r["s"], t0)
    emit("  busy per stream: " + ", ".join(f"{k} {v / 100:.0f} us ({v / (t1 - t0):.0%})" for k, v in sorted(busy.items())))
    chain, cur = [nxt], nxt
    while True:
        # the binding dependency: of the launch's graph dependencies (own-stream predecessor, waited-on
        # streams' launches), the one that finished last
        cands = [q for q in deps.get(cur["i"], []) if q["e"] > t0 and q["s"]]
        if not cands:
            break
        p = max(cands, key=lambda r: r["e"])
        chain.append(p)
        if p is first or p["s"] <= t0:
            break
        cur = p
    chain.reverse()
    ktime = sum(r["e"] - r["s"] for r in chain if r["s"] >= t0 and r is not nxt)
    emit(f"  critical chain (from the captured graph's edges: own-stream order + the logged cross-stream waits; "
         f"each step back the dependency that finished last): {len(chain)} launches, {ktime / 100:.0f} us of "
         f"kernels + {(t1 - t0 - ktime) / 100:.0f} us between them (launch gaps, unstamped kernels)")
    for r in chain:
        emit(f"    {r['stream']:>8} {(r['s'] - t0) / 100:8.1f} {(r['e'] - t0) / 100:8.1f} {(r['e'] - r['s']) / 100:7.1f}  {r['tag']}")
if a.list:
    rx = re.compile(a.list)
    for r in recs:
        if rx.search(r["tag"]):
            emit(f"  {r['stream']:>8} {(r['s'] - t_first) / 100:10.1f} {(r['e'] - r['s']) / 100:7.1f}  {r['tag']}")
if a.out:
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        f.write("\n".join(out) + "\n")
