#!/bin/bash
# round 4: build LDS-cap A/B, then an in-situ pass that prefers fewer split-K passes at equal step time
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_r4f.sh || exit 1
PY_TIMEOUT=1000 PY_TAIL=60 PY_ARGS="--alts-only --top 40 --reps 10 --prefer-nosplit 0.002 --match (h30_w40|h60_w80|h120_w160) --try 19:1 20:1 21:1 23:1 3:1 4:1 5:1 35:1 36:1 37:1 40:1 41:1 43:1 24:1 25:1 27:1 28:1 --out gpurun_out/r4/tune_insitu3.json" \
  bash tools/gpu_r4.sh py:tools/insitu_tune.py
