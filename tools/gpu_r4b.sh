#!/bin/bash
# round 4, in-situ search of the new tiles over the cfg2 step (tools/insitu_tune.py --try)
PY_TIMEOUT=1100 PY_TAIL=80 PY_ARGS="--alts-only --top 45 --reps 10 --try 43:1 43:2 11:1 27:1 27:2 28:1 28:2 29:1 29:2 30:1 --out gpurun_out/r4/tune_insitu2.json" \
  bash tools/gpu_r4.sh py:tools/insitu_tune.py
