#!/bin/bash
# GPU call: the volume tiles 8/9 once (were refused after a fault), range tests, full GPU suite, bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-range}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "conv3d_halo_vs_torch" -x -q --timeout 120 --timeout-method thread > $OUT/t3d.log 2>&1 || { echo "3d rc=$?"; tail -30 $OUT/t3d.log; exit 1; }
tail -2 $OUT/t3d.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "range" -x -q --timeout 120 --timeout-method thread > $OUT/trange.log 2>&1 || { echo "range rc=$?"; tail -30 $OUT/trange.log; exit 1; }
tail -2 $OUT/trange.log
FSMI_PARITY_LOG=$OUT/parity.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $OUT/tall.log 2>&1 || { echo "all rc=$?"; tail -30 $OUT/tall.log; exit 1; }
tail -2 $OUT/tall.log; cat $OUT/parity.jsonl
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 > $OUT/b_$i.json 2>>$OUT/b.err || { echo "bench rc=$?"; tail -5 $OUT/b.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/b_$i.json')); print('bench', round(d['value'],3), round(d['ms_per_step'],2), 'conv frac', round(d['roofline_conv']['frac'],3))"
done
