#!/usr/bin/env python3
"""One-line summary of a bench.py JSON line (the last line of FILE)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline", {})
b = d.get("roofline_build", {})
c = d.get("roofline_conv", {})
cs = d.get("roofline_conv_step", {})
p = d.get("parity", {})


def f(x, n=3):
    return None if x is None else round(x, n)


print(json.dumps({"value": f(d["value"]), "ms": f(d["ms_per_step"], 2), "n_gpus": d.get("n_gpus"),
                  "world": d.get("world_size"), "lk_frac": f(r.get("frac")), "lk_us": f(r.get("avg_us"), 1),
                  "lk_single_us": f(r.get("avg_us_single_stream", r.get("avg_us_kernel_clock")), 1),
                  "build_frac": f(b.get("frac")), "conv": f(c.get("frac")), "conv_step": f(cs.get("frac")),
                  "dd": p.get("max_abs_dd_px"), "overflow": d.get("range_overflow")}))
