#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) per fsmi kernel.

    python tools/pmc_summary.py gpurun_out/round [--config cfg2 --corr-levels 4] > profiles/...

Per MI355X_MICROARCH.md §HBM: both counters are in KB; on gfx950 FETCH_SIZE
tallies each 128-B memory-side read request as 64 B, so it is doubled here
(the lookup's 4-B-per-lane loads of 64 consecutive floats issue 128-B
requests like a wide stream); WRITE_SIZE is taken as is.  Each counter comes
from its own profiling pass.  Writes profiles/pmc_lookup_summary.json (read
by bench.py for `roofline.traffic`) and prints a per-kernel table.
"""
import argparse
import collections
import csv
import json
import os
import re

ap = argparse.ArgumentParser()
ap.add_argument("round_dir")
ap.add_argument("--config", default="cfg2")
ap.add_argument("--corr-levels", type=int, default=4)
ap.add_argument("--pairs-per-gpu", type=int, default=1)
ap.add_argument("--out", default="profiles/pmc_lookup_summary.json")
a = ap.parse_args()

per = collections.defaultdict(dict)
for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
    path = os.path.join(a.round_dir, f"pmc_{ctr}", "pmc_counter_collection.csv")
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = re.sub(r"\(.*", "", r["Kernel_Name"].replace("fsmi::(anonymous namespace)::", "").replace("void ", ""))
        vals[name].append(float(r["Counter_Value"]))
    for k, v in vals.items():
        per[k][ctr] = sum(v) / len(v)
        per[k]["launches_" + ctr] = len(v)

rows = {}
print(f"{'kernel':34s} {'FETCH_SIZE KB':>14s} {'x2 (gfx950)':>12s} {'WRITE_SIZE KB':>14s} {'HBM MB/launch':>14s}")
for k, d in sorted(per.items()):
    f, w = d.get("FETCH_SIZE", 0.0), d.get("WRITE_SIZE", 0.0)
    hbm = (2 * f + w) * 1024
    rows[k] = {"fetch_kb_raw": f, "write_kb": w, "hbm_bytes_per_launch": hbm}
    print(f"{k:34s} {f:14.1f} {2 * f:12.1f} {w:14.1f} {hbm / 1e6:14.2f}")

lk = [k for k in rows if k.startswith("geo_lookup_kernel")]
summary = {"config": a.config, "corr_levels": a.corr_levels, "pairs_per_gpu": a.pairs_per_gpu,
           "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), {a.round_dir}",
           "correction": "FETCH_SIZE x2 (gfx950 128-B requests tallied at 64 B), KB -> B x1024",
           "hbm_bytes_per_launch": rows[lk[0]]["hbm_bytes_per_launch"] if lk else None,
           "build_hbm_bytes_per_launch": next((v["hbm_bytes_per_launch"] for k, v in rows.items()
                                               if k.startswith("build_stem_kernel")), None),
           "kernels": rows}
os.makedirs(os.path.dirname(a.out), exist_ok=True)
with open(a.out, "w") as fh:
    json.dump(summary, fh, indent=1)
