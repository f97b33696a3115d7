#!/usr/bin/env python3
"""Per-kernel table of a rocprofv3 --kernel-trace --stats run directory (the *kernel_stats.csv in it).

    python tools/stats_brief.py gpurun_out/r4/trace_cfg2 [--top 25] [--per N]

--per N divides the totals by N (e.g. the forwards the command ran) for per-forward milliseconds.
"""
import argparse
import csv
import glob
import os
import re

ap = argparse.ArgumentParser()
ap.add_argument("run_dir")
ap.add_argument("--top", type=int, default=25)
ap.add_argument("--per", type=float, default=0.0)
a = ap.parse_args()
paths = [a.run_dir] if os.path.isfile(a.run_dir) else glob.glob(os.path.join(a.run_dir, "**", "*kernel_stats.csv"), recursive=True)
if not paths:
    raise SystemExit(f"no kernel_stats.csv under {a.run_dir}")
rows = list(csv.DictReader(open(paths[0])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)


def short(n):
    n = n.replace("fsmi::(anonymous namespace)::", "").replace("fsmi::halo::", "").replace("void ", "")
    return re.sub(r"\((fsmi|float|int|const|HaloArgs).*", "", n)[:90]


print(f"{paths[0]}  total {tot / 1e6:.2f} ms")
print(f"{'calls':>6} {'avg_us':>9} {'total_ms':>9} {'pct':>6}  kernel")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:a.top]:
    t = float(r["TotalDurationNs"])
    print(f"{int(r['Calls']):>6} {float(r['AverageNs']) / 1e3:>9.2f} {t / 1e6 / (a.per or 1):>9.3f} "
          f"{100 * t / tot:>6.2f}  {short(r['Name'])}")
