#!/bin/bash
# GPU call: new GPU tests (world-2 real model, autocast), then an A/B of split-K on small maps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ab_split; mkdir -p $OUT
FSMI_PARITY_LOG=$OUT/parity.jsonl timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_configs.py -k "world2 or autocast" -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/tests.log; exit 1; }
tail -4 $OUT/tests.log; cat $OUT/parity.jsonl
for i in 1 2; do
  for mp in 0 4800 1200; do
    FSMI_SPLIT_MAXPIX=$mp timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 > $OUT/b_${mp}_$i.json 2>>$OUT/b.err || { echo "bench rc=$?"; tail -5 $OUT/b.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$OUT/b_${mp}_$i.json')); print('maxpix $mp run $i', round(d['value'],3), round(d['ms_per_step'],2))"
  done
done
