#!/bin/bash
# round 3, call AC: build kernel with the two-half overlapped staging -- parity tests, A/B against the
# one-phase schedule (FSMI_BUILD_DBG bit 3), cfg2 bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r3ac
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "comb or build or e2e or lookup or geo" --timeout 250 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for r in 1 2; do
timeout -k 10 180 python tools/build_bench.py --dbg 0 8 16 24 1 2 --tiles "" > $OUT/build$r.txt 2>&1 || { echo "build rc=$?"; tail -5 $OUT/build$r.txt; exit 1; }
cat $OUT/build$r.txt
done
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -5 $OUT/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print('cfg2', round(d['value'],3), round(d['ms_per_step'],2), 'build', round(d['roofline_build']['frac'],4), round(d['roofline_build']['avg_us'],2))"
echo done-r3ac
