#!/bin/bash
# Round profile on the GPU box: default bench line, rocprofv3 kernel-trace stats of
# the same command, and PMC passes (FETCH_SIZE, WRITE_SIZE) for the fsmi kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/round
rm -rf $OUT; mkdir -p $OUT
ARGS="--steps ${STEPS:-5} --warmup 2 $BENCH_ARGS"
timeout -k 10 600 python3 bench.py $ARGS > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -5 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS --no-cpu-baseline > $OUT/trace_bench.json 2> $OUT/trace.err || { echo "trace rc=$?"; tail -5 $OUT/trace.err; exit 1; }
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $ctr --kernel-include-regex 'fsmi' --output-format csv -d $OUT/pmc_$ctr -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline $BENCH_ARGS > $OUT/pmc_$ctr.json 2> $OUT/pmc_$ctr.err || { echo "pmc $ctr rc=$?"; tail -5 $OUT/pmc_$ctr.err; exit 1; }
done
ls -R $OUT | head -40
