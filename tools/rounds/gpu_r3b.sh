#!/bin/bash
# round 3, call B: range + reference-order GPU tests, guard A/B bench, conv PMC on the top loop layers
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r3b
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_range.py tests/test_gpu_reference_order.py -m gpu -x -v --timeout 500 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 300 python tools/reference_order_bench.py --config cfg2 > $OUT/refbench.json 2> $OUT/refbench.err || { echo "refbench rc=$?"; tail -5 $OUT/refbench.err; exit 1; }
cat $OUT/refbench.json
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $OUT/bench_guard_$i.json 2> $OUT/bench_guard_$i.err || { echo "bench rc=$?"; tail -5 $OUT/bench_guard_$i.err; exit 1; }
FSMI_RANGE_GUARD=0 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $OUT/bench_noguard_$i.json 2> $OUT/bench_noguard_$i.err || { echo "bench rc=$?"; tail -5 $OUT/bench_noguard_$i.err; exit 1; }
done
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r3b/bench_*.json")):
    d=json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"],3), round(d["ms_per_step"],2), round(d["roofline"]["frac"],3), round(d["roofline_conv"]["frac"],3), d.get("range_recoveries"))
PY
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE"
for L in gru04.conv1 gru04.conv0 gru04.zr_l gru04.q_l enc.convc2 enc.convc1; do
  i=0
  for P in "$P1" "$P2" "FETCH_SIZE"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $P --kernel-include-regex 'conv_' --output-format csv -d $OUT/pmc_${L}_$i -o pmc -- python3 tools/conv_bench.py --mode halo --no-miopen --reps 3 --only $L > $OUT/pmc_${L}_$i.log 2>&1 || { echo "pmc $L $i rc=$?"; tail -5 $OUT/pmc_${L}_$i.log; exit 1; }
  done
done
echo pmc-done
