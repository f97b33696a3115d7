#!/bin/bash
# pointwise-tile parity, then a tuning pass of the 2D 1x1 shapes with the pointwise candidates
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "pw" > gpurun_out/pw_tests.log 2>&1 || { tail -40 gpurun_out/pw_tests.log; exit 1; }
tail -2 gpurun_out/pw_tests.log
timeout -k 10 600 python -u tools/tune_conv.py --config cfg2 --only-cfgs 24 25 26 --match "^k1_d1_" --reps 10 \
  > gpurun_out/tune_pw.txt 2> gpurun_out/tune_pw.err || { tail -20 gpurun_out/tune_pw.err; exit 1; }
cat gpurun_out/tune_pw.txt
mkdir -p gpurun_out/tuning && cp tuning/fsmi_conv.json gpurun_out/tuning/
