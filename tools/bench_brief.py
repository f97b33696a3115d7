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
g = d.get("roofline_build_lookup", {})
m = d.get("allpairs_mfma", {})


def f(x, n=3):
    return None if x is None else round(x, n)


print(json.dumps({"value": f(d["value"]), "ms": f(d["ms_per_step"], 2), "n_gpus": d.get("n_gpus"),
                  "world": d.get("world_size"), "lk_frac": f(r.get("frac")), "lk_us": f(r.get("avg_us"), 1),
                  "lk_single_us": f(r.get("avg_us_single_stream", r.get("avg_us_kernel_clock")), 1),
                  "build_frac": f(b.get("frac")), "build_us": f(b.get("avg_us"), 1),
                  "build_replay_frac": f(b.get("frac_replay")), "geo_frac": f(g.get("frac")),
                  "geo_us_pair": f(g.get("us_per_pair"), 1), "geo_kernels_us": g.get("per_kernel_us"),
                  "ap_mfma": f(m.get("frac")), "ap_us": f(m.get("avg_us"), 1),
                  "conv": f(c.get("frac")), "conv_step": f(cs.get("frac")),
                  "dd": p.get("max_abs_dd_px"), "overflow": d.get("range_overflow")}))
