#!/bin/bash
# graph-timed re-tune of every cfg2 conv shape (all candidates), then pw_bench for reference
set -o pipefail
mkdir -p gpurun_out/tuning
timeout -k 10 300 python -u tools/pw_bench.py > gpurun_out/pw_bench_graph.txt 2>&1 || { tail -20 gpurun_out/pw_bench_graph.txt; exit 1; }
cat gpurun_out/pw_bench_graph.txt | cut -c1-300
timeout -k 10 1000 python -u tools/tune_conv.py --config cfg2 --reps 10 > gpurun_out/retune_cfg2.txt 2> gpurun_out/retune_cfg2.err || { tail -20 gpurun_out/retune_cfg2.err; exit 1; }
tail -2 gpurun_out/retune_cfg2.err
cp tuning/fsmi_conv.json gpurun_out/tuning/
