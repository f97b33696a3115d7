#!/bin/bash
# round 3, call F: re-tune cfg2/cfg3 shapes with the pipelined (32+c) and depth (30) tiles, A/B bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r3f
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 900 python tools/tune_conv.py --config cfg2 cfg3 --only-cfgs 30 34 35 36 37 38 39 40 41 --out $OUT/fsmi_conv.json > $OUT/tune.jsonl 2> $OUT/tune.err || { echo "tune rc=$?"; tail -5 $OUT/tune.err; exit 1; }
tail -2 $OUT/tune.err
for i in 1 2; do
FSMI_TUNE_PATH=$OUT/fsmi_conv.json timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $OUT/bench_new_$i.json 2> $OUT/bench_new_$i.err || { echo "bench rc=$?"; tail -5 $OUT/bench_new_$i.err; exit 1; }
FSMI_TUNE_PATH=tuning/ab/fsmi_conv_r2.json timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $OUT/bench_old_$i.json 2> $OUT/bench_old_$i.err || { echo "bench rc=$?"; tail -5 $OUT/bench_old_$i.err; exit 1; }
done
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r3f/bench_*.json")):
    d=json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"],3), round(d["ms_per_step"],2), round(d["roofline"]["frac"],3), round(d["roofline_conv"]["frac"],3), d.get("range_overflow"))
PY
