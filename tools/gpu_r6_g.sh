# round-6 GPU step G: in-situ retune of the cfg2 step after the context-part hoist (new conv shapes), then a
# same-box A/B of the committed table vs the retuned one (three alternating rounds)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r6g
mkdir -p $O
timeout -k 10 700 python -u tools/insitu_tune.py --config cfg2 --top 20 --out $O/fsmi_conv.json > $O/insitu.txt 2>&1 || exit $?
[ -f $O/fsmi_conv.json ] || cp tuning/fsmi_conv.json $O/fsmi_conv.json
ab() {   # ab NAME ENV...
  local name=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/ab_$name.json 2> $O/ab_$name.err || return $?
  python -c "import json; d=json.load(open('$O/ab_$name.json')); print('$name', round(d['value'], 3), 'pairs/s', round(d['ms_per_step'], 2), 'ms')" >> $O/ab.txt
}
for r in 1 2 3; do
  ab committed_r$r || exit $?
  ab insitu_r$r FSMI_TUNE_PATH=$O/fsmi_conv.json || exit $?
done
cat $O/ab.txt
