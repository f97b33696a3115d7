#!/bin/bash
# Memory-path PMC for one conv layer/config: L1 (TCP) -> L2 (TCC) request volume, L2 hit rate,
# TA busy/stall cycles.  LAYER3D=1 runs tools/conv3d_bench.py shapes instead of the 2D ones.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/conv_mem_${TAG:-x}
rm -rf $OUT; mkdir -p $OUT
P1="TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
P2="TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"
P3="TCP_PENDING_STALL_CYCLES_sum TD_BUSY_sum TCP_TCC_READ_REQ_LATENCY_sum GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-include-regex 'conv_halo' --output-format csv -d $OUT/p$i -o pmc -- python3 tools/conv_bench.py --mode halo --no-miopen --reps 3 --only $LAYER --cfg ${CFG:--1} > $OUT/p$i.log 2>&1 || { echo "pmc pass $i rc=$?"; tail -5 $OUT/p$i.log; exit 1; }
done
echo ok
