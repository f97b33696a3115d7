#!/bin/bash
# stride-2 2D (context net) tiles: op + block + end-to-end parity, then bench A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "s2 or resblock or context or e2e or golden or hier or replay or batch" > gpurun_out/s2ctx_tests.log 2>&1 || { tail -40 gpurun_out/s2ctx_tests.log; exit 1; }
tail -2 gpurun_out/s2ctx_tests.log
bash tools/gpu_ab_env.sh FSMI_S2=0
