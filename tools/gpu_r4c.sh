#!/bin/bash
# round 4 profile set: cfg2 bench + rocprof kernel stats of the same command + FETCH/WRITE PMC + SQ
# counters, cfg3 bench + its kernel stats
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_r4.sh bench trace pmc sq bench3 trace3 || exit 1
python3 tools/iter_timeline.py gpurun_out/r4/trace_cfg2 > gpurun_out/r4/iter_timeline_cfg2.txt
head -3 gpurun_out/r4/iter_timeline_cfg2.txt
