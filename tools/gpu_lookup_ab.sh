#!/bin/bash
# lookup variants (FSMI_LIB), interleaved rounds: LIBS="default nt ..."
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for v in $LIBS; do
    if [ "$v" = "default" ]; then L=foundationstereo_amd/_lib/libfsmi.so; else L=foundationstereo_amd/_lib/libfsmi_$v.so; fi
    FSMI_LIB=$L timeout -k 10 120 python -u tools/lookup_bench.py 2>>gpurun_out/lookup_ab.err || { echo "lookup $v rc=$?"; tail -5 gpurun_out/lookup_ab.err; exit 1; }
  done
done
