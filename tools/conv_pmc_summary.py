#!/usr/bin/env python3
"""Summarise rocprofv3 SQ counter passes per kernel: MFMA pipe utilisation, instruction mix, LDS
bank conflicts, resident waves.

    python tools/conv_pmc_summary.py gpurun_out/r3w --passes pmc_P1 pmc_P2 [--top 12] [--out profiles/x.json]

Pass P1 = SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES
SQ_WAVES GRBM_GUI_ACTIVE; pass P2 = SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT
SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE (each its own run: rocprofv3 does not
split counters over passes).  Units per MI355X_MICROARCH.md: GRBM_GUI_ACTIVE is summed over the 8
XCDs (kernel cycles = value / 8); SQ_VALU_MFMA_BUSY_CYCLES counts MFMA-pipe cycles summed over SIMDs
(32 per v_mfma_f32_32x32x16_f16), so

    mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)

is the fraction of the chip's MFMA issue capacity the kernel used over its own duration (the 3xfp16
split issues three MFMAs per fp32-equivalent product, so the fp32-equivalent rate is a third of it).
SQ_WAVE_CYCLES / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY count quad-cycles; waves_per_simd =
4 * SQ_WAVE_CYCLES / (cycles * 1024).
"""
import argparse
import collections
import csv
import json
import os
import re

ap = argparse.ArgumentParser()
ap.add_argument("round_dir")
ap.add_argument("--passes", nargs="+", default=["pmc_P1", "pmc_P2"])
ap.add_argument("--top", type=int, default=12)
ap.add_argument("--match", default="", help="regex on the kernel name")
ap.add_argument("--out", default="")
a = ap.parse_args()


def short(name):
    n = name.replace("fsmi::(anonymous namespace)::", "").replace("fsmi::halo::", "").replace("void ", "")
    return re.sub(r"\((fsmi|float|int|const|HaloArgs).*", "", n)


ctr = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for p in a.passes:
    path = os.path.join(a.round_dir, p, "pmc_counter_collection.csv")
    seen = set()
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        if a.match and not re.search(a.match, k):
            continue
        ctr[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        key = (p, r["Dispatch_Id"])
        if key not in seen:
            seen.add(key)
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)

rows = []
for k, c in ctr.items():
    m = {n: sum(v) / len(v) for n, v in c.items()}
    cyc = m.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
    us = sum(dur[k]) / len(dur[k])
    launches = max(len(v) for v in c.values()) // max(1, sum(1 for p in a.passes))
    row = {"kernel": k, "launches_per_pass": launches, "avg_us": round(us, 2), "total_ms": round(us * launches / 1e3, 3)}
    if cyc > 0:
        row["clock_ghz"] = round(cyc / us / 1e3, 2)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            row["mfma_busy"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024), 3)
        if "SQ_WAVE_CYCLES" in m:
            row["waves_per_simd"] = round(4 * m["SQ_WAVE_CYCLES"] / (cyc * 1024), 2)
            if "SQ_WAIT_INST_ANY" in m:
                row["wait_inst_frac"] = round(m["SQ_WAIT_INST_ANY"] / m["SQ_WAVE_CYCLES"], 3)
            if "SQ_ACTIVE_INST_ANY" in m:
                row["issue_frac"] = round(m["SQ_ACTIVE_INST_ANY"] / m["SQ_WAVE_CYCLES"], 3)
    mf = m.get("SQ_INSTS_MFMA", 0.0)
    if mf > 0:
        row["mfma_insts"] = int(mf)
        for n, lab in (("SQ_INSTS_VALU", "valu_per_mfma"), ("SQ_INSTS_LDS", "lds_per_mfma"),
                       ("SQ_INSTS_SALU", "salu_per_mfma"), ("SQ_INSTS_VMEM_RD", "vmem_rd_per_mfma")):
            if n in m:
                row[lab] = round(m[n] / mf, 2)
    if m.get("SQ_LDS_IDX_ACTIVE", 0.0) > 0:
        row["lds_bank_conflict"] = round(m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"], 4)
    rows.append(row)
rows.sort(key=lambda r: -r["total_ms"])
rows = rows[:a.top]
cols = ["avg_us", "total_ms", "clock_ghz", "mfma_busy", "waves_per_simd", "issue_frac", "wait_inst_frac",
        "valu_per_mfma", "lds_per_mfma", "lds_bank_conflict"]
print(f"{'kernel':60s} " + " ".join(f"{c[:10]:>10s}" for c in cols))
for r in rows:
    print(f"{r['kernel'][:60]:60s} " + " ".join(f"{r.get(c, ''):>10}" for c in cols))
if a.out:
    with open(a.out, "w") as fh:
        json.dump({"source": f"rocprofv3 --pmc passes {a.passes} under {a.round_dir}",
                   "formulae": "mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * 1024); "
                               "waves_per_simd = 4*SQ_WAVE_CYCLES / (GRBM_GUI_ACTIVE/8 * 1024)",
                   "kernels": rows}, fh, indent=1)
