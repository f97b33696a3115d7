#!/bin/bash
# round 4: pipelined-tile triple weight buffer A/B (default W3 vs the libfsmi_w2.so variant), then the
# persistent-build A/B at cfg3
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TEST_PATHS="tests/test_gpu_pipe.py" bash tools/gpu_r4.sh test || exit 1
AB_ENVS="FSMI_LIB=foundationstereo_amd/_lib/libfsmi_w2.so;FSMI_W3=1" AB_REPS=3 bash tools/gpu_r4.sh ab || exit 1
bash tools/gpu_r4d.sh
