#!/bin/bash
# round 3, call A: full GPU suite, smoke, cfg2 bench with / without the per-forward range guard
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r3a
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $OUT/bench_guard_$i.json 2> $OUT/bench_guard_$i.err || { echo "bench rc=$?"; tail -5 $OUT/bench_guard_$i.err; exit 1; }
FSMI_RANGE_GUARD=0 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $OUT/bench_noguard_$i.json 2> $OUT/bench_noguard_$i.err || { echo "bench rc=$?"; tail -5 $OUT/bench_noguard_$i.err; exit 1; }
done
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r3a/bench_*.json")):
    d=json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"],3), d["ms_per_step"], d["roofline"]["frac"], d["roofline_conv"]["frac"], d.get("range_recoveries"))
PY
