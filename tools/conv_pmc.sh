#!/bin/bash
# PMC passes over the halo conv kernel on one layer shape (stall breakdown, LDS conflicts).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/conv_pmc
rm -rf $OUT; mkdir -p $OUT
LAYER=${LAYER:-gru04.conv1}
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVES"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-include-regex 'conv_halo' --output-format csv -d $OUT/p$i -o pmc -- python3 tools/conv_bench.py --mode halo --no-miopen --reps 3 --only $LAYER --cfg ${CFG:--1} > $OUT/p$i.log 2>&1 || { echo "pmc pass $i rc=$?"; tail -5 $OUT/p$i.log; exit 1; }
done
echo ok
