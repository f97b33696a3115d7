#!/bin/bash
# GPU call: selected tests (PYTEST_SEL) + N bench runs (BENCH_N, default 2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-quick}; mkdir -p $OUT
if [ -n "$PYTEST_SEL" ]; then
  FSMI_PARITY_LOG=$OUT/parity.jsonl timeout -k 10 900 python -u -m pytest $PYTEST_SEL -x -q --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $OUT/tests.log; exit 1; }
  tail -2 $OUT/tests.log; cat $OUT/parity.jsonl 2>/dev/null
fi
for i in $(seq 1 ${BENCH_N:-2}); do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 $BENCH_ARGS > $OUT/b_$i.json 2>>$OUT/b.err || { echo "bench rc=$?"; tail -5 $OUT/b.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/b_$i.json')); print('bench', round(d['value'],3), round(d['ms_per_step'],2), 'conv frac', round(d['roofline_conv']['frac'],3), 'lookup frac', round(d['roofline']['frac'],3))"
done
