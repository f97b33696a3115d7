#!/bin/bash
# fused lookup conv: parity tests (op + end to end), then the bench with and without the fusion
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "lookup or e2e or update or golden" > gpurun_out/fuse_tests.log 2>&1 || { tail -40 gpurun_out/fuse_tests.log; exit 1; }
tail -2 gpurun_out/fuse_tests.log
bash tools/gpu_ab_env.sh FSMI_FUSE_LOOKUP=0
