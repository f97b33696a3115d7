#!/bin/bash
# full GPU suite + smoke, then a library A/B on the bench (LIBS)
set -o pipefail
mkdir -p gpurun_out
( while true; do date > gpurun_out/heartbeat; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/full_tests.log 2>&1 || { tail -40 gpurun_out/full_tests.log; exit 1; }
tail -2 gpurun_out/full_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full_smoke.log 2>&1 || { tail -20 gpurun_out/full_smoke.log; exit 1; }
tail -1 gpurun_out/full_smoke.log
if [ -n "$LIBS" ]; then ROUNDS=${ROUNDS:-3} TAG=abfull bash tools/gpu_ab_libs.sh; fi
