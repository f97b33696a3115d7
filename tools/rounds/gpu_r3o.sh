#!/bin/bash
# round 3, call O: B prefetch in every register-weight tile -- full GPU suite, bench, re-tune A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r3o
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; grep -v MIOpen $OUT/tests.log | tail -30; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 900 python tools/tune_conv.py --config cfg2 cfg3 --only-cfgs 3 4 5 6 7 8 9 19 20 21 23 34 35 36 37 38 39 40 41 --match '_d1_.*_D1_' --out $OUT/fsmi_conv.json > $OUT/tune.jsonl 2> $OUT/tune.err || { echo "tune rc=$?"; tail -5 $OUT/tune.err; exit 1; }
tail -1 $OUT/tune.err
for i in 1 2 3; do
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $OUT/bench_base_$i.json 2> $OUT/bench_base_$i.err || { echo "bench rc=$?"; tail -5 $OUT/bench_base_$i.err; exit 1; }
FSMI_TUNE_PATH=$OUT/fsmi_conv.json timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $OUT/bench_new_$i.json 2> $OUT/bench_new_$i.err || { echo "bench rc=$?"; tail -5 $OUT/bench_new_$i.err; exit 1; }
done
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r3o/bench_*.json")):
    d=json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"],3), round(d["ms_per_step"],2), round(d["roofline"]["frac"],3), round(d["roofline_conv"]["frac"],3))
PY
