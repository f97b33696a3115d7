#!/bin/bash
# full GPU parity suite, smoke, then the default bench twice
set -o pipefail
mkdir -p gpurun_out
# heartbeat: the full-size CPU-oracle tests print nothing for minutes
( while true; do date > gpurun_out/heartbeat; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/check_tests.log 2>&1 || { tail -40 gpurun_out/check_tests.log; exit 1; }
tail -2 gpurun_out/check_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/check_smoke.log 2>&1 || { tail -20 gpurun_out/check_smoke.log; exit 1; }
tail -1 gpurun_out/check_smoke.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/check_bench_$r.json 2> gpurun_out/check_bench_$r.err || { tail -20 gpurun_out/check_bench_$r.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/check_bench_$r.json').read().strip().splitlines()[-1]);print(round(d['value'],3), round(d['ms_per_step'],2), d['roofline']['frac'], d.get('roofline_conv',{}).get('frac'))"
done
