#!/bin/bash
# round 3, call W: classifier direct conv (8-deep depth-fastest tile) parity + timing, cfg2 bench,
# SQ counter passes (MFMA busy, instruction mix) over the bench's fsmi kernels, classifier traffic
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r3w
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "conv3d_direct or e2e or classifier" --timeout 250 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 120 python tools/tile_ab.py --set cls > $OUT/cls.jsonl 2> $OUT/cls.err || { echo "cls rc=$?"; tail -5 $OUT/cls.err; exit 1; }
cat $OUT/cls.jsonl
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -5 $OUT/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_conv']['frac'])"
P1="SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-include-regex 'fsmi' --output-format csv -d $OUT/pmc_P$i -o pmc -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/pmc_P$i.json 2> $OUT/pmc_P$i.err || { echo "pmc P$i rc=$?"; tail -5 $OUT/pmc_P$i.err; exit 1; }
done
python3 tools/conv_pmc_summary.py $OUT --top 16 --out $OUT/sq_summary_cfg2.json > $OUT/sq_table.txt
cat $OUT/sq_table.txt
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-include-regex 'conv3d_direct|allpairs|conv_depth' --output-format csv -d $OUT/pmc_$ctr -o pmc -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/pmc_$ctr.json 2> $OUT/pmc_$ctr.err || { echo "pmc $ctr rc=$?"; tail -5 $OUT/pmc_$ctr.err; exit 1; }
done
python3 tools/pmc_summary.py $OUT --out $OUT/pmc_cls.json
echo done-r3w
