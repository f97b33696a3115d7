#!/bin/bash
# round 3, call G: A/B bench of tuning tables (r2 vs r3a merged)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r3g
rm -rf $OUT; mkdir -p $OUT
for i in 1 2 3; do
for t in r3a r2; do
FSMI_TUNE_PATH=tuning/ab/fsmi_conv_$t.json timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $OUT/bench_${t}_$i.json 2> $OUT/bench_${t}_$i.err || { echo "bench rc=$?"; tail -5 $OUT/bench_${t}_$i.err; exit 1; }
done
done
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r3g/bench_*.json")):
    d=json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"],3), round(d["ms_per_step"],2), round(d["roofline"]["frac"],3), round(d["roofline_conv"]["frac"],3), d.get("range_overflow"))
PY
