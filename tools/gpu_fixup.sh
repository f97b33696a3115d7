#!/bin/bash
# split-K fixup A/B: parity of the split / volume / e2e tests, then cfg2 bench with and without it
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "halo or e2e or conv3d or update" > gpurun_out/fixup_tests.log 2>&1 || { tail -30 gpurun_out/fixup_tests.log; exit 1; }
tail -3 gpurun_out/fixup_tests.log
for r in 1 2; do
  timeout -k 10 180 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/fixup_on_$r.json 2> gpurun_out/fixup_on_$r.err || exit 1
  FSMI_HALO_FIXUP=0 timeout -k 10 180 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/fixup_off_$r.json 2> gpurun_out/fixup_off_$r.err || exit 1
done
for f in gpurun_out/fixup_o*_?.json; do echo "$f $(python -c "import json,sys;d=json.loads(open('$f').read().strip().splitlines()[-1]);print(round(d['value'],3), round(d['ms_per_step'],2))")"; done
