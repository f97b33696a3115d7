# round-6 GPU step K: in-situ search of the chain's big 3x3 convs (gru04 conv1 / zr / q, convc2) over tiles that
# fit one round of blocks beside the pipeline stream (256 x 5 rows, split-K 1 / 2), then a same-box A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r6k
mkdir -p $O
timeout -k 10 700 python -u tools/insitu_tune.py --config cfg2 --top 12 --alts 2 --match 'k3_d1_ci(512|256)_co(512|256|128)_b1_D1_h120_w160' \
  --try 43:1 43:2 41:1 41:2 40:2 40:4 19:1 19:2 --out $O/fsmi_conv.json > $O/insitu.txt 2>&1 || exit $?
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
