#!/usr/bin/env python3
"""Per-kernel statistics of ONE step out of a rocprofv3 kernel trace database (rocpd SQLite, the
``*_results.db`` that ``rocprofv3 --kernel-trace --stats -d DIR -o NAME`` writes on this image).

A step is the window between two consecutive starts of ``--anchor`` (a kernel launched once per step,
default the cost-volume build ``build_stem``); the last complete window is reported (``--window -2`` for
the one before, ...).  Prints the window span, the summed kernel time, and per kernel name: launches,
total / average us and share, sorted by total; ``--csv`` also writes them as CSV.

    python tools/rocpd_stats.py gpurun_out/r6s/prof_bb/bb_results.db [--anchor build_stem] [--csv out.csv]
"""
import argparse
import collections
import csv
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--anchor", default="build_stem")
    ap.add_argument("--window", type=int, default=-1)
    ap.add_argument("--csv", default="")
    ap.add_argument("--top", type=int, default=60)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, grid_x, grid_y, grid_z, workgroup_x from kernels order by start").fetchall()
    starts = [r[1] for r in rows if a.anchor in r[0]]
    assert len(starts) >= 2, f"anchor {a.anchor!r} found {len(starts)} times"
    print("anchor windows (us):", " ".join(f"{(e - s) / 1e3:.0f}" for s, e in zip(starts, starts[1:])))
    t0, t1 = starts[a.window - 1], starts[a.window]
    win = [r for r in rows if t0 <= r[1] < t1]
    per = collections.defaultdict(lambda: [0, 0])
    for name, s, e, *_ in win:
        short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        per[short][0] += 1
        per[short][1] += e - s
    busy = sum(v[1] for v in per.values())
    print(f"window {a.window} between '{a.anchor}' starts: span {(t1 - t0) / 1e3:.1f} us, "
          f"{len(win)} launches, summed kernel time {busy / 1e3:.1f} us")
    items = sorted(per.items(), key=lambda kv: -kv[1][1])
    print(f"{'kernel':70s} {'calls':>6s} {'total_us':>10s} {'avg_us':>9s} {'share':>6s}")
    for k, (n, tot) in items[:a.top]:
        print(f"{k[:70]:70s} {n:6d} {tot / 1e3:10.1f} {tot / 1e3 / n:9.2f} {100 * tot / busy:5.1f}%")
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
            for k, (n, tot) in items:
                w.writerow([k, n, tot, tot / n, 100 * tot / busy])


if __name__ == "__main__":
    main()
