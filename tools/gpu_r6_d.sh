# round-6 GPU check D: same-box cfg2 A/Bs of the loop split with its partial sums on the pipeline stream
# (FSMI_LOOP_PRE), the Cout=1 head kernel (FSMI_COUT1) and the convq split (FSMI_Q_SPLIT, opt-in), then the
# replay timeline of the default
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r6d
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ctx_pre.py tests/test_gpu_capture_fork.py -q -x --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || exit $?
ab() {   # ab NAME ENV...
  local name=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/ab_$name.json 2> $O/ab_$name.err || return $?
  python -c "import json; d=json.load(open('$O/ab_$name.json')); print('$name', round(d['value'], 3), 'pairs/s', round(d['ms_per_step'], 2), 'ms')" >> $O/ab.txt
}
for r in 1 2 3; do
  ab loop1_r$r || exit $?
  ab loop0_r$r FSMI_LOOP_PRE=0 || exit $?
  ab cout0_r$r FSMI_COUT1=0 || exit $?
done
ab qsplit1 FSMI_Q_SPLIT=1 || exit $?
cat $O/ab.txt
timeout -k 10 300 python -u tools/replay_timeline.py --out $O/replay_timeline.txt > $O/replay_timeline.log 2>&1
