#!/usr/bin/env python3
"""One refinement iteration of a graph-REPLAYED forward from a rocprofv3 kernel trace, with its
hardware queues and the chain of kernels that sets the iteration's length.

    python tools/step_timeline.py gpurun_out/r5/trace_cfg2 [--forward -2] [--iter 16] [--iters 32]

bench.py's traced command runs warmup forwards (eager), the timed replays of the captured forward
(4 streams -> several hardware queues) and, last, one single-stream EAGER pass for its per-kernel
event timing.  ``--forward -2`` (default) selects the last timed replay; ``-1`` would be that
serialised eager pass.  For iteration ``--iter`` (lookup(t) start .. lookup(t+1) start) it prints
every dispatch with queue, start / end (us from lookup(t)), duration and grid, the busy time per
queue, the time two or more queues run kernels at once, and the critical chain: starting from
lookup(t+1), repeatedly the kernel that finished last before the current one started (any queue)
-- the dependency the current kernel waited for, as far as the trace shows it.
"""
import argparse
import csv
import glob
import os
import re

ap = argparse.ArgumentParser()
ap.add_argument("run_dir")
ap.add_argument("--forward", type=int, default=-2, help="which forward (-1 = last traced)")
ap.add_argument("--iter", type=int, default=16)
ap.add_argument("--iters", type=int, default=32)
ap.add_argument("--quiet", action="store_true", help="summary and chain only")
a = ap.parse_args()
path = glob.glob(os.path.join(a.run_dir, "**", "*kernel_trace.csv"), recursive=True)[0]
rows = list(csv.DictReader(open(path)))
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
rows.sort(key=lambda r: r["s"])
lk = [i for i, r in enumerate(rows) if "geo_lookup" in r["Kernel_Name"]]
base = len(lk) + a.forward * a.iters
first, nxt = lk[base + a.iter], lk[base + a.iter + 1]
t0, t1 = rows[first]["s"], rows[nxt]["s"]


def short(n):
    n = n.replace("fsmi::(anonymous namespace)::", "").replace("fsmi::halo::", "").replace("void ", "")
    return re.sub(r"\((fsmi|float|int|const|HaloArgs|LookupArgs|MlpArgs).*", "", n)[:58]


sel = [r for r in rows if r["e"] > t0 and r["s"] < t1]
queues = sorted({r["Queue_Id"] for r in sel}, key=int)
print(f"forward {a.forward}, iteration {a.iter}: span {(t1 - t0) / 1e3:.1f} us (lookup to lookup), "
      f"{len(sel)} dispatches on queues {queues}")
if not a.quiet:
    for r in sel:
        s, e = (r["s"] - t0) / 1e3, (r["e"] - t0) / 1e3
        g = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        print(f"  q{r['Queue_Id']:>2} {s:8.1f} {e:8.1f} {e - s:7.1f}  grid {g:>6}  {short(r['Kernel_Name'])}")
# busy time per queue, and overlap (time with >= 2 queues busy)
ev = []
for r in sel:
    ev.append((max(r["s"], t0), 1, r["Queue_Id"]))
    ev.append((min(r["e"], t1), -1, r["Queue_Id"]))
ev.sort()
busy = {q: 0 for q in queues}
active = {q: 0 for q in queues}
multi = any_busy = 0
prev = t0
for t, d, q in ev:
    n_active = sum(1 for v in active.values() if v > 0)
    for qq, v in active.items():
        if v > 0:
            busy[qq] += t - prev
    if n_active >= 2:
        multi += t - prev
    if n_active >= 1:
        any_busy += t - prev
    active[q] += d
    prev = t
span = t1 - t0
print("  busy per queue: " + ", ".join(f"q{q} {busy[q] / 1e3:.0f} us ({busy[q] / span:.0%})" for q in queues)
      + f"; some queue busy {any_busy / span:.0%}, two or more {multi / span:.0%}")
# critical chain backward from lookup(t+1)
chain = [rows[nxt]]
cur = rows[nxt]
while True:
    cands = [r for r in rows if r["e"] <= cur["s"] and r["e"] > t0 - 1 and r is not cur]
    if not cands:
        break
    p = max(cands, key=lambda r: r["e"])
    chain.append(p)
    if p is rows[first] or p["s"] <= t0:
        break
    cur = p
chain.reverse()
tot = sum(r["e"] - r["s"] for r in chain if r["s"] >= t0)
gaps = span - tot
print(f"  critical chain (last finisher before each start): {len(chain)} kernels, {tot / 1e3:.0f} us of kernels "
      f"+ {gaps / 1e3:.0f} us of gaps")
by_q = {}
for r in chain:
    by_q[r["Queue_Id"]] = by_q.get(r["Queue_Id"], 0) + (r["e"] - r["s"])
print("  chain time by queue: " + ", ".join(f"q{q} {v / 1e3:.0f} us" for q, v in sorted(by_q.items(), key=lambda x: int(x[0]))))
for r in chain:
    s, e = (r["s"] - t0) / 1e3, (r["e"] - t0) / 1e3
    print(f"    q{r['Queue_Id']:>2} {s:8.1f} {e:8.1f} {e - s:7.1f}  {short(r['Kernel_Name'])}")
