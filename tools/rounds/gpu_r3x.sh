#!/bin/bash
# round 3, call X (re-entry sanity): full GPU suite + smoke + cfg2 bench on the restored tree
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r3x
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py --steps 20 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -5 $OUT/bench.err; exit 1; }
cat $OUT/bench.json

timeout -k 10 180 python tools/build_bench.py --dbg 0 1 2 3 --tiles "" 8,12 10,12 20,6 > $OUT/build.txt 2>&1 || { echo "build rc=$?"; tail -5 $OUT/build.txt; exit 1; }
cat $OUT/build.txt
timeout -k 10 180 python tools/lookup_bench.py > $OUT/lookup.txt 2>&1 || { echo "lookup rc=$?"; tail -5 $OUT/lookup.txt; exit 1; }
cat $OUT/lookup.txt

timeout -k 10 300 python bench.py --precision fast --steps 20 > $OUT/bench_fast.json 2> $OUT/bench_fast.err || { echo "bench fast rc=$?"; tail -5 $OUT/bench_fast.err; exit 1; }
cat $OUT/bench_fast.json
echo done-r3x
