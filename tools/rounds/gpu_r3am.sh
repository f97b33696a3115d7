#!/bin/bash
# round 3, call AM: cfg4 and cfg5 (hierarchical) bench lines with the final code
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r3am
rm -rf $OUT; mkdir -p $OUT
for c in cfg4 cfg5; do
timeout -k 10 400 python bench.py --config $c --no-cpu-baseline --steps 5 > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { echo "$c rc=$?"; tail -5 $OUT/bench_$c.err; exit 1; }
tail -1 $OUT/bench_$c.json
done
echo done-r3am
