#!/bin/bash
# late round-2 final: parity subset for the last changes, then the cfg2 and cfg3 round profiles
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "s2 or resblock or e2e or golden or hier or replay or batch or autocast" > gpurun_out/final2_tests.log 2>&1 || { tail -40 gpurun_out/final2_tests.log; exit 1; }
tail -2 gpurun_out/final2_tests.log
CONFIG=cfg2 bash tools/gpu_round_profile.sh || exit 1
CONFIG=cfg3 PPG=4 bash tools/gpu_round_profile.sh || exit 1
