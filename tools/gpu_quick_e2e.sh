#!/bin/bash
# end-to-end parity subset, then three default bench runs (the first on a warmed box)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py \
  -k "e2e or golden or hier or replay or batch or autocast or hourglass or cfg" > gpurun_out/quick_tests.log 2>&1 || { tail -40 gpurun_out/quick_tests.log; exit 1; }
tail -2 gpurun_out/quick_tests.log
bash tools/gpu_ab_env.sh FSMI_CTX_OVERLAP=0
