#!/bin/bash
# round 3, call AB = AA (pipelined depth conv: tests, tile A/B, cfg2 bench) then Z (lookup CPC A/B,
# geometry SQ counters, fast-precision kernel stats)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/rounds/gpu_r3aa.sh || exit 1
bash tools/rounds/gpu_r3z.sh || exit 1
