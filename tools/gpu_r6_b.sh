# round-6 GPU check B: the hoisted conv0 context part (update.SelectiveConvGRU.context_pre, act 7):
# its tests, tuning of the new conv shapes (cfg2 .. cfg5, new keys only) and a same-box cfg2 A/B
# FSMI_CTX_PRE=1 / 0 (alternating, three rounds) on the tuned table
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r6b
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ctx_pre.py -q -x --timeout 300 --timeout-method thread > $O/ctx_pre_tests.txt 2>&1 || exit $?
timeout -k 10 500 python -u tools/tune_conv.py --config cfg2 cfg3 cfg4 cfg5 --new-only --out $O/fsmi_conv.json > $O/tune.txt 2>&1 || exit $?
export FSMI_TUNE_PATH=$O/fsmi_conv.json
for r in 1 2 3; do
  for on in 1 0; do
    FSMI_CTX_PRE=$on timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/ab_ctx${on}_r$r.json 2> $O/ab_ctx${on}_r$r.err || exit $?
    python -c "import json,sys; d=json.load(open('$O/ab_ctx${on}_r$r.json')); print('ctx_pre=$on round $r', round(d['value'], 3), 'pairs/s', round(d['ms_per_step'], 2), 'ms')" >> $O/ab.txt
  done
done
cat $O/ab.txt
