#!/usr/bin/env python3
"""Timeline of one refinement iteration from a rocprofv3 kernel trace: every dispatch between two
consecutive geo_lookup launches of the LAST traced forward, with start / end relative to the first
lookup, its hardware queue and duration.

    python tools/iter_timeline.py gpurun_out/r4/trace_cfg2 [--iter 16]
"""
import argparse
import csv
import glob
import os
import re

ap = argparse.ArgumentParser()
ap.add_argument("run_dir")
ap.add_argument("--iter", type=int, default=16, help="iteration of the last forward (0-based)")
ap.add_argument("--iters", type=int, default=32)
a = ap.parse_args()
path = glob.glob(os.path.join(a.run_dir, "**", "*kernel_trace.csv"), recursive=True)[0]
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
lk = [i for i, r in enumerate(rows) if "geo_lookup" in r["Kernel_Name"]]
first = lk[-a.iters + a.iter]
nxt = lk[-a.iters + a.iter + 1]
t0 = int(rows[first]["Start_Timestamp"])
t_end = int(rows[nxt]["Start_Timestamp"])


def short(n):
    n = n.replace("fsmi::(anonymous namespace)::", "").replace("fsmi::halo::", "").replace("void ", "")
    return re.sub(r"\((fsmi|float|int|const|HaloArgs|LookupArgs).*", "", n)[:60]


sel = [r for r in rows if int(r["End_Timestamp"]) > t0 and int(r["Start_Timestamp"]) < t_end]
print(f"iteration span {(t_end - t0) / 1e3:.1f} us (lookup to lookup)")
for r in sel:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"q{r['Queue_Id']:>3} {s / 1e3:8.1f} {e / 1e3:8.1f} {(e - s) / 1e3:7.1f}  grid {int(r['Grid_Size_X']) // int(r['Workgroup_Size_X']):>5}  {short(r['Kernel_Name'])}")
