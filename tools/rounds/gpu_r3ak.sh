#!/bin/bash
# round 3, call AK: final cfg2 round profile and cfg3 / fast bench lines with the final bench.py
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r3ak
rm -rf $OUT; mkdir -p $OUT
CONFIG=cfg2 bash tools/gpu_round_profile.sh || exit 1
timeout -k 10 300 python bench.py --config cfg3 --no-cpu-baseline --steps 5 > $OUT/bench_cfg3.json 2> $OUT/bench_cfg3.err || { echo "cfg3 rc=$?"; tail -5 $OUT/bench_cfg3.err; exit 1; }
tail -1 $OUT/bench_cfg3.json
timeout -k 10 300 python bench.py --precision fast --steps 20 > $OUT/bench_fast.json 2> $OUT/bench_fast.err || { echo "fast rc=$?"; tail -5 $OUT/bench_fast.err; exit 1; }
tail -1 $OUT/bench_fast.json
echo done-r3ak
