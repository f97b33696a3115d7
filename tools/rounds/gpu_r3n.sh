#!/bin/bash
# round 3, call N: re-tune the 2D shapes over the pipelined tiles, A/B bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r3n
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 900 python tools/tune_conv.py --config cfg2 cfg3 --only-cfgs 34 35 36 37 38 39 40 41 --match '_d1_.*_D1_' --out $OUT/fsmi_conv.json > $OUT/tune.jsonl 2> $OUT/tune.err || { echo "tune rc=$?"; tail -5 $OUT/tune.err; exit 1; }
tail -1 $OUT/tune.err
for i in 1 2 3; do
FSMI_TUNE_PATH=$OUT/fsmi_conv.json timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $OUT/bench_new_$i.json 2> $OUT/bench_new_$i.err || { echo "bench rc=$?"; tail -5 $OUT/bench_new_$i.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $OUT/bench_base_$i.json 2> $OUT/bench_base_$i.err || { echo "bench rc=$?"; tail -5 $OUT/bench_base_$i.err; exit 1; }
done
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r3n/bench_*.json")):
    d=json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"],3), round(d["ms_per_step"],2), round(d["roofline"]["frac"],3), round(d["roofline_conv"]["frac"],3))
PY
