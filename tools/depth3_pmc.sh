#!/bin/bash
# SQ counter passes over the 3^3 volume conv of cfg2's stem (tools/depth3_bench.py --only stem: the
# table's tile and cfg 31), one rocprofv3 --pmc run per pass; summary: tools/conv_pmc_summary.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/depth3_pmc
rm -rf $OUT; mkdir -p $OUT
P1="SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE"
P3="SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_IFETCH SQ_INST_CYCLES_VMEM SQ_WAVE_CYCLES SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex 'conv_' --output-format csv -d $OUT/pmc_P$i -o pmc -- \
    python3 tools/depth3_bench.py --only stem > $OUT/p$i.log 2>&1 || { echo "pmc pass $i rc=$?"; tail -5 $OUT/p$i.log; exit 1; }
done
# instruction-fetch / wait counters: a pass of its own, not fatal (counter names vary by ROCm release)
timeout -s KILL 120 rocprofv3 --pmc $P3 --kernel-include-regex 'conv_' --output-format csv -d $OUT/pmc_P3 -o pmc -- \
  python3 tools/depth3_bench.py --only stem > $OUT/p3.log 2>&1 || { echo "pmc pass 3 rc=$?"; tail -3 $OUT/p3.log; }
python3 tools/conv_pmc_summary.py $OUT --top 8 --out $OUT/sq.json > $OUT/sq_table.txt; python3 tools/pmc_generic.py $OUT >> $OUT/sq_table.txt; cat $OUT/sq_table.txt
