#!/bin/bash
# round 3, call Y: 4-pixel-per-lane lookup (geo_lookup_v4_kernel) -- bit-exact vs the scalar kernel,
# lookup micro-bench A/B, cfg2 / cfg3 bench lines with it
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r3y
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "lookup or geo" --timeout 250 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for v in 0 1 0 1; do
FSMI_LOOKUP_V4=$v timeout -k 10 180 python tools/lookup_bench.py >> $OUT/lookup_v$v.txt 2>&1 || { echo "lookup rc=$?"; tail -5 $OUT/lookup_v$v.txt; exit 1; }
done
tail -n 2 $OUT/lookup_v*.txt
for v in 1 0; do
FSMI_LOOKUP_V4=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $OUT/bench_v$v.json 2> $OUT/bench_v$v.err || { echo "bench rc=$?"; tail -5 $OUT/bench_v$v.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench_v$v.json').read().strip().splitlines()[-1]); print('cfg2 v$v', round(d['value'],3), round(d['ms_per_step'],2), round(d['roofline']['frac'],4), d['roofline']['avg_us'])"
done
for v in 1 0; do
FSMI_LOOKUP_V4=$v timeout -k 10 300 python bench.py --config cfg3 --no-cpu-baseline --steps 5 > $OUT/bench3_v$v.json 2> $OUT/bench3_v$v.err || { echo "bench3 rc=$?"; tail -5 $OUT/bench3_v$v.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench3_v$v.json').read().strip().splitlines()[-1]); print('cfg3 v$v', round(d['value'],3), round(d['ms_per_step'],2), round(d['roofline']['frac'],4), d['roofline']['avg_us'])"
done
echo done-r3y
