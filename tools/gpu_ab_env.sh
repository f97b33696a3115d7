#!/bin/bash
# A/B of environment knobs on the default bench: bash tools/gpu_ab_env.sh "FSMI_SPLIT_CAP=1" "FSMI_SPLIT_CAP=2" ...
set -o pipefail
mkdir -p gpurun_out
run() {
  env $1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]);print('$1', round(d['value'],3), round(d['ms_per_step'],2))"
}
# one unreported run first: the first bench on a fresh box runs slow (clocks / caches warming up)
env FSMI_NONE=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > /dev/null 2>&1
for r in 1 2 3; do
  run "FSMI_NONE=1"
  for k in "$@"; do run "$k"; done
done
