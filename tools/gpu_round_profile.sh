#!/bin/bash
# Round profile on the GPU box for CONFIG (default cfg2): the bench line, a rocprofv3 kernel-trace
# stats pass of the same command, and PMC passes (FETCH_SIZE, WRITE_SIZE, one per run) over the
# fsmi kernels summarised into profiles-style JSON (tools/pmc_summary.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
CONFIG=${CONFIG:-cfg2}
OUT=gpurun_out/round_$CONFIG
rm -rf $OUT; mkdir -p $OUT
ARGS="--config $CONFIG --steps ${STEPS:-5} --warmup 2 $BENCH_ARGS"
timeout -k 10 600 python3 bench.py $ARGS > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -5 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS --no-cpu-baseline > $OUT/trace_bench.json 2> $OUT/trace.err || { echo "trace rc=$?"; tail -5 $OUT/trace.err; exit 1; }
if [ -z "$NO_PMC" ]; then
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $ctr --kernel-include-regex 'fsmi' --output-format csv -d $OUT/pmc_$ctr -o pmc -- python3 bench.py --config $CONFIG --steps 2 --warmup 1 --no-cpu-baseline $BENCH_ARGS > $OUT/pmc_$ctr.json 2> $OUT/pmc_$ctr.err || { echo "pmc $ctr rc=$?"; tail -5 $OUT/pmc_$ctr.err; exit 1; }
done
python3 tools/pmc_summary.py $OUT --config $CONFIG --pairs-per-gpu ${PPG:-1} --out $OUT/pmc_lookup_summary_$CONFIG.json > $OUT/pmc_table.txt
fi
echo profiled $CONFIG
