# round-6 GPU step J: gru16(t+1) enqueued after gru04(t) (FSMI_GRU16_LATE) vs beside it, same-box cfg2 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r6j
mkdir -p $O
ab() {   # ab NAME ENV...
  local name=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/ab_$name.json 2> $O/ab_$name.err || return $?
  python -c "import json; d=json.load(open('$O/ab_$name.json')); print('$name', round(d['value'], 3), 'pairs/s', round(d['ms_per_step'], 2), 'ms')" >> $O/ab.txt
}
for r in 1 2 3; do
  ab base_r$r || exit $?
  ab late_r$r FSMI_GRU16_LATE=1 || exit $?
done
cat $O/ab.txt
