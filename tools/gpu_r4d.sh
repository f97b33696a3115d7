#!/bin/bash
# round 4: persistent build A/B at cfg3 (bench line + rocprof kernel stats per arm)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r4
AB_CONFIG=cfg3 AB_ENVS="FSMI_BUILD_PERSIST=0;FSMI_BUILD_PERSIST=1" AB_REPS=1 STEPS=10 bash tools/gpu_r4.sh ab || exit 1
for p in 0 1; do
  rm -rf $OUT/trace_persist$p
  FSMI_BUILD_PERSIST=$p timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_persist$p -o run -- \
    python3 bench.py --config cfg3 --steps 5 --warmup 3 --no-cpu-baseline > $OUT/trace_persist$p.json 2> $OUT/trace_persist$p.err || { echo "trace $p failed"; tail -5 $OUT/trace_persist$p.err; exit 1; }
  python3 tools/stats_brief.py $OUT/trace_persist$p --top 60 | grep -i "build_stem\|total"
done
