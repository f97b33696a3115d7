#!/bin/bash
# Bench (N=1) then a rocprofv3 kernel-trace profile of the same command, on the GPU box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
STEPS=${STEPS:-5}
timeout -k 10 600 python3 bench.py --steps $STEPS --warmup 2 $BENCH_ARGS > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed rc=$?"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
if [ -n "$PROF" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline $BENCH_ARGS > $OUT/prof_bench.json 2> $OUT/prof.err || { echo "prof failed rc=$?"; tail -20 $OUT/prof.err; exit 1; }
  find $OUT/prof -name "*stats*" | head
fi
