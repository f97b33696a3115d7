# round-6 GPU step L: the one-round 80-pixel EdgeNeXt MLP tile (FSMI_MLP_PX=80) re-measured now that the
# disparity head is on the iteration's critical chain: its test, then a 4-round same-box cfg2 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r6l
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp80.py -q -x --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || exit $?
ab() {   # ab NAME ENV...
  local name=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/ab_$name.json 2> $O/ab_$name.err || return $?
  python -c "import json; d=json.load(open('$O/ab_$name.json')); print('$name', round(d['value'], 3), 'pairs/s', round(d['ms_per_step'], 2), 'ms')" >> $O/ab.txt
}
for r in 1 2 3 4; do
  ab px64_r$r || exit $?
  ab px80_r$r FSMI_MLP_PX=80 || exit $?
done
cat $O/ab.txt
