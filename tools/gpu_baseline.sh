#!/bin/bash
# One GPU call: parity tests, smoke, the default bench line and a rocprofv3 kernel-stats pass of it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-base}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $OUT/gpu_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 300 python -u bench.py ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -5 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
[ -n "$NO_PROF" ] && exit 0
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --no-cpu-baseline ${BENCH_ARGS} > $OUT/trace_bench.json 2> $OUT/trace.err || { echo "trace rc=$?"; tail -5 $OUT/trace.err; exit 1; }
echo traced
