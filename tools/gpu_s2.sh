#!/bin/bash
# stride-2 tiles + fused FeatureAtt gate: op parity, end-to-end parity, micro-bench, then the bench A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "s2 or gate or hourglass or up2 or e2e or golden or hier or batch or replay or filter3d" > gpurun_out/s2_tests.log 2>&1 || { tail -40 gpurun_out/s2_tests.log; exit 1; }
tail -2 gpurun_out/s2_tests.log
timeout -k 10 300 python -u tools/s2_bench.py > gpurun_out/s2_bench.log 2>&1 || { tail -20 gpurun_out/s2_bench.log; exit 1; }
cat gpurun_out/s2_bench.log
bash tools/gpu_ab_env.sh "FSMI_S2=0 FSMI_FATT=0" FSMI_FATT=0
