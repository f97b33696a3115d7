#!/bin/bash
# round 3, call AH (final): full GPU suite + smoke, then the round profile of cfg2 (bench line,
# rocprofv3 kernel stats, FETCH / WRITE PMC passes) and cfg3 / cfg2-fast bench lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r3ah
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/tests.log; exit 1; }
tail -6 $OUT/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
CONFIG=cfg2 bash tools/gpu_round_profile.sh || exit 1
timeout -k 10 300 python bench.py --config cfg3 --no-cpu-baseline --steps 5 > $OUT/bench_cfg3.json 2> $OUT/bench_cfg3.err || { echo "cfg3 rc=$?"; tail -5 $OUT/bench_cfg3.err; exit 1; }
tail -1 $OUT/bench_cfg3.json
timeout -k 10 300 python bench.py --precision fast --steps 20 > $OUT/bench_fast.json 2> $OUT/bench_fast.err || { echo "fast rc=$?"; tail -5 $OUT/bench_fast.err; exit 1; }
tail -1 $OUT/bench_fast.json
echo done-r3ah
