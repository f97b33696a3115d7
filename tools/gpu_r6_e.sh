# round-6 GPU check E: the convq split (FSMI_Q_SPLIT) without the loop split, same-box cfg2 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r6e
mkdir -p $O
ab() {   # ab NAME ENV...
  local name=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/ab_$name.json 2> $O/ab_$name.err || return $?
  python -c "import json; d=json.load(open('$O/ab_$name.json')); print('$name', round(d['value'], 3), 'pairs/s', round(d['ms_per_step'], 2), 'ms')" >> $O/ab.txt
}
for r in 1 2 3; do
  ab base_r$r FSMI_LOOP_PRE=0 || exit $?
  ab qsplit_r$r FSMI_LOOP_PRE=0 FSMI_Q_SPLIT=1 || exit $?
  ab cout0_r$r FSMI_LOOP_PRE=0 FSMI_COUT1=0 || exit $?
done
cat $O/ab.txt
