#!/bin/bash
# transposed-conv phase tiles: op parity, end-to-end parity, then the bench with / without them
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "up2 or e2e or golden or hier or batch or replay" > gpurun_out/up_tests.log 2>&1 || { tail -40 gpurun_out/up_tests.log; exit 1; }
tail -2 gpurun_out/up_tests.log
bash tools/gpu_ab_env.sh FSMI_UP3D=0
