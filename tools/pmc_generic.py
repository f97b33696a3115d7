#!/usr/bin/env python3
"""Average every PMC counter per kernel over the rocprofv3 passes under a directory.

    python tools/pmc_generic.py gpurun_out/build_pmc [--match build_stem]

Counters are summed over the dispatch's dimensions (rocprofv3 reports one row per counter per
dispatch) and averaged over dispatches.  Raw units: SQ_* cycle counters in quad-cycles,
FETCH_SIZE / WRITE_SIZE in KB (FETCH_SIZE x2 on gfx950, MI355X_MICROARCH.md §HBM).
"""
import argparse
import collections
import csv
import glob
import os
import re

ap = argparse.ArgumentParser()
ap.add_argument("root")
ap.add_argument("--match", default="")
a = ap.parse_args()
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sorted(glob.glob(os.path.join(a.root, "**", "*counter_collection.csv"), recursive=True)):
    per_dispatch = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        name = re.sub(r"\(.*", "", r["Kernel_Name"].replace("fsmi::(anonymous namespace)::", "").replace("void ", ""))
        if a.match and a.match not in name:
            continue
        per_dispatch[(name, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (name, _, ctr), v in per_dispatch.items():
        vals[name][ctr].append(v)
for name, ctrs in sorted(vals.items()):
    print(name)
    for ctr, v in sorted(ctrs.items()):
        print(f"  {ctr:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
