#!/bin/bash
# round 4: build LDS cap A/B (one block per CU vs two), cfg3 and cfg2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
AB_CONFIG=cfg3 AB_ENVS="FSMI_BUILD_LDS_KB=160;FSMI_BUILD_LDS_KB=80" AB_REPS=2 STEPS=10 bash tools/gpu_r4.sh ab || exit 1
AB_CONFIG=cfg2 AB_ENVS="FSMI_BUILD_LDS_KB=160;FSMI_BUILD_LDS_KB=80" AB_REPS=2 bash tools/gpu_r4.sh ab || exit 1
