# round-6 GPU check C: gru04's conv0 / conv1 split off the chain (FSMI_LOOP_PRE), convq split by inputs
# (FSMI_Q_SPLIT) and DispHead's Cout=1 kernel (FSMI_COUT1): tests incl. the captured fork patterns and full-size parity, tuning of the new shapes, same-box
# cfg2 A/Bs on the tuned table, then the replay timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r6c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ctx_pre.py tests/test_gpu_capture_fork.py tests/test_gpu_configs.py \
  "tests/test_gpu_parity.py::test_conv3x3_cout1_vs_torch" "tests/test_gpu_parity.py::test_e2e_vs_oracle" \
  "tests/test_gpu_parity.py::test_e2e_vs_reference_golden" "tests/test_gpu_parity.py::test_graph_replay_matches_eager" "tests/test_gpu_parity.py::test_selective_gru_fused_vs_oracle" "tests/test_gpu_parity.py::test_update_step_golden" \
  -q -x --timeout 400 --timeout-method thread > $O/tests.txt 2>&1 || exit $?
timeout -k 10 500 python -u tools/tune_conv.py --config cfg2 cfg3 cfg4 cfg5 --new-only --out $O/fsmi_conv.json > $O/tune.txt 2>&1 || exit $?
export FSMI_TUNE_PATH=$O/fsmi_conv.json
ab() {   # ab NAME ENV...
  local name=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/ab_$name.json 2> $O/ab_$name.err || return $?
  python -c "import json; d=json.load(open('$O/ab_$name.json')); print('$name', round(d['value'], 3), 'pairs/s', round(d['ms_per_step'], 2), 'ms')" >> $O/ab.txt
}
for r in 1 2; do
  ab all_r$r || exit $?
  ab loop0_r$r FSMI_LOOP_PRE=0 || exit $?
  ab qsplit0_r$r FSMI_Q_SPLIT=0 || exit $?
  ab cout0_r$r FSMI_COUT1=0 || exit $?
done
cat $O/ab.txt
timeout -k 10 300 python -u tools/replay_timeline.py --out $O/replay_timeline.txt > $O/replay_timeline.log 2>&1
