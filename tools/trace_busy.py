#!/usr/bin/env python3
"""Busy / overlap analysis of a rocprofv3 kernel trace over the bench's timed graph replays.

    python tools/trace_busy.py gpurun_out/.../run_kernel_trace.csv [--last-steps 3]

Splits the trace into forwards at the geo_lookup bursts (32 per forward), takes the last N
forwards, and reports: wall time, GPU busy time (union of kernel intervals), idle gaps, mean
kernel concurrency, and per-kernel-family busy share -- whether the step is throughput-bound
(GPU always busy) or latency-bound (gaps on the critical path)."""
import argparse
import collections
import csv
import re

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--last-steps", type=int, default=3)
a = ap.parse_args()
rows = []
for r in csv.DictReader(open(a.trace)):
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r["Queue_Id"])))
rows.sort()
lk = [i for i, r in enumerate(rows) if "geo_lookup" in r[2]]
# forwards: groups of 32 lookups; a forward starts at the first kernel after the previous forward's
# last lookup + its tail; use lookup index boundaries
n_fwd = len(lk) // 32
starts = [lk[32 * f] for f in range(n_fwd)]
ends = [lk[32 * f + 31] for f in range(n_fwd)]
sel = range(max(0, n_fwd - a.last_steps), n_fwd)
fam = collections.Counter()
tot_wall = tot_busy = tot_sum = 0
for f in sel:
    # window: from the end of the previous forward's last lookup to the end of this one's
    lo = rows[ends[f - 1]][1] if f > 0 else rows[0][0]
    hi = rows[ends[f]][1] + 2_000_000      # + 2 ms for the post-loop tail (upsample)
    if f + 1 < n_fwd:
        hi = min(hi, rows[starts[f + 1]][0])
    iv = [(s, e, n) for s, e, n, q in rows if s >= lo and s < hi]
    iv.sort()
    busy = 0
    cur_s, cur_e = None, None
    for s, e, n in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    ksum = sum(e - s for s, e, n in iv)
    wall = max(e for s, e, n in iv) - min(s for s, e, n in iv)
    tot_wall += wall
    tot_busy += busy
    tot_sum += ksum
    for s, e, n in iv:
        m = re.search(r"::(\w+?)(<|\()", n)
        fam[m.group(1) if m else n[:40]] += e - s
    print(f"forward {f}: wall {wall / 1e6:.2f} ms  busy {busy / 1e6:.2f} ms ({100 * busy / wall:.1f} %)  "
          f"kernel-sum {ksum / 1e6:.2f} ms  concurrency {ksum / busy:.2f}  kernels {len(iv)}")
print(f"mean: wall {tot_wall / len(sel) / 1e6:.2f} ms, busy {100 * tot_busy / tot_wall:.1f} %, "
      f"concurrency {tot_sum / tot_busy:.2f}")
for k, v in fam.most_common(15):
    print(f"  {k:40s} {v / len(sel) / 1e6:8.2f} ms  {100 * v / tot_sum:5.1f} %")
