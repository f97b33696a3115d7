#!/bin/bash
# GPU steps, one parametrised script (output under $GPU_OUT, default gpurun_out/r5).
#   bash tools/gpu_steps.sh STEP [STEP ...]
# Steps:
#   test        pytest -m gpu (per-test timeout, stops at the first failure; TEST_PATHS, TEST_K = a -k expression)
#   bench       bench.py cfg2 (20 steps) -> bench_cfg2.json
#   bench3      bench.py cfg3 -> bench_cfg3.json
#   trace       rocprofv3 --kernel-trace --stats of the cfg2 bench command
#   trace3      the same for cfg3
#   pmc         FETCH_SIZE / WRITE_SIZE passes (one counter per run) + tools/pmc_summary.py, cfg2
#   sq          SQ_ counters (MFMA busy, instruction mix) over the conv kernels, cfg2
#   smoke       __graft_entry__.smoke()
#   ab          A/B of environment settings on the bench (AB_ENVS="K=V;K=V2", AB_REPS rounds)
#   py:<file>   python3 <file> (a tool script), output to <file base>.out
# Every GPU step runs under its own timeout and the script stops at the first failing step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=${GPU_OUT:-gpurun_out/r5}
mkdir -p $OUT
BENCH_ARGS=${BENCH_ARGS:-}
fail() { echo "$1 rc=$2"; tail -20 "$3"; exit 1; }
for step in "$@"; do
  echo "== $step $(date +%T)"
  case $step in
    test)
      KARGS=(); [ -n "${TEST_K:-}" ] && KARGS=(-k "$TEST_K")
      timeout -k 10 1100 python3 -u -m pytest ${TEST_PATHS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread ${TEST_ARGS:-} "${KARGS[@]}" \
        > $OUT/test.log 2>&1 || fail test $? $OUT/test.log
      tail -3 $OUT/test.log ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || fail smoke $? $OUT/smoke.log
      tail -2 $OUT/smoke.log ;;
    bench|bench3|bench4|bench5)
      cfg=cfg2; [ $step = bench3 ] && cfg=cfg3; [ $step = bench4 ] && cfg=cfg4; [ $step = bench5 ] && cfg=cfg5
      timeout -k 10 400 python3 bench.py --config $cfg --steps ${STEPS:-20} --warmup 5 $BENCH_ARGS \
        > $OUT/bench_$cfg.json 2> $OUT/bench_$cfg.err || fail bench $? $OUT/bench_$cfg.err
      python3 tools/bench_brief.py $OUT/bench_$cfg.json ;;
    trace|trace3)
      cfg=cfg2; [ $step = trace3 ] && cfg=cfg3
      rm -rf $OUT/trace_$cfg
      timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$cfg -o run -- \
        python3 bench.py --config $cfg --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline $BENCH_ARGS \
        > $OUT/trace_bench_$cfg.json 2> $OUT/trace_$cfg.err || fail trace $? $OUT/trace_$cfg.err
      python3 tools/bench_brief.py $OUT/trace_bench_$cfg.json
      python3 tools/stats_brief.py $OUT/trace_$cfg --top 25 > $OUT/trace_$cfg.txt && head -40 $OUT/trace_$cfg.txt ;;
    pmc)
      for ctr in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 300 rocprofv3 --pmc $ctr --kernel-include-regex 'fsmi' --output-format csv -d $OUT/pmc_$ctr -o pmc -- \
          python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline $BENCH_ARGS > $OUT/pmc_$ctr.json 2> $OUT/pmc_$ctr.err \
          || fail "pmc $ctr" $? $OUT/pmc_$ctr.err
      done
      python3 tools/pmc_summary.py $OUT --config cfg2 --pairs-per-gpu 1 --out $OUT/pmc_lookup_summary_cfg2.json > $OUT/pmc_table.txt
      cat $OUT/pmc_table.txt | head -30 ;;
    sq)
      P1="SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"
      P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE"
      i=0
      for P in "$P1" "$P2"; do
        i=$((i+1))
        timeout -s KILL 300 rocprofv3 --pmc $P --kernel-include-regex 'fsmi' --output-format csv -d $OUT/pmc_P$i -o pmc -- \
          python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline $BENCH_ARGS > $OUT/pmc_P$i.json 2> $OUT/pmc_P$i.err \
          || fail "sq P$i" $? $OUT/pmc_P$i.err
      done
      python3 tools/conv_pmc_summary.py $OUT --top 16 --out $OUT/sq_cfg2.json > $OUT/sq_table.txt
      cat $OUT/sq_table.txt ;;
    ab)
      # A/B of environment settings on the cfg2 bench: AB_ENVS="K=V K2=V2;K=V3" (';' separates the arms),
      # AB_REPS rounds of every arm in turn
      IFS=';' read -ra ARMS <<< "${AB_ENVS}"
      for r in $(seq 1 ${AB_REPS:-2}); do
        for i in "${!ARMS[@]}"; do
          arm="${ARMS[$i]}"
          timeout -k 10 300 env $arm python3 bench.py --config ${AB_CONFIG:-cfg2} --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline $BENCH_ARGS \
            > $OUT/ab_${i}_$r.json 2> $OUT/ab_${i}_$r.err || fail "ab arm $i" $? $OUT/ab_${i}_$r.err
          echo "arm $i [$arm] round $r: $(python3 tools/bench_brief.py $OUT/ab_${i}_$r.json)"
        done
      done ;;
    py:*)
      f=${step#py:}; b=$(basename $f .py)
      timeout -k 10 ${PY_TIMEOUT:-400} python3 -u $f ${PY_ARGS:-} > $OUT/$b.out 2> $OUT/$b.err || fail "$f" $? $OUT/$b.err
      tail -${PY_TAIL:-40} $OUT/$b.out ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "done $(date +%T)"
