#!/bin/bash
# PMC passes over the single-pass build kernel (tools/build_bench.py, one tile), one counter
# group per rocprofv3 run (gpurun refuses oversized groups); summaries -> gpurun_out/build_pmc/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/build_pmc
rm -rf $OUT; mkdir -p $OUT
ARGS="--reps 5 --tiles ${TILE:-8,12}"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE" "TA_BUSY_avr TA_BUSY_max"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-include-regex 'build_stem' --output-format csv -d $OUT/p$i -o pmc -- python3 tools/build_bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_generic.py $OUT --match build_stem > $OUT/summary.txt 2>&1 || true
cat $OUT/summary.txt | head -40
