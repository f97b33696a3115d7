#!/bin/bash
# round 3, call Q: cfg3 / cfg4 / cfg5 round profiles (bench line, kernel-trace stats, FETCH/WRITE PMC)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for C in cfg4 cfg5 cfg3; do
  PPG=1; [ $C = cfg3 ] && PPG=4
  CONFIG=$C PPG=$PPG STEPS=5 BENCH_ARGS="--no-cpu-baseline" timeout -k 10 1000 bash tools/gpu_round_profile.sh > gpurun_out/prof_$C.log 2>&1 || { echo "$C rc=$?"; tail -5 gpurun_out/prof_$C.log; exit 1; }
  tail -2 gpurun_out/prof_$C.log
done
