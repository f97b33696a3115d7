#!/bin/bash
# round 3, call AI: in-situ re-tune of the cfg2 table over the current kernels (top shapes by share
# of the step, splits up to 2 plus each shape's current tile unsplit); merged table to gpurun_out
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r3ai
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 1000 python -u tools/insitu_tune.py --config cfg2 --top 14 --max-split 2 --nosplit --write --out $OUT/fsmi_conv.json > $OUT/insitu.jsonl 2> $OUT/insitu.err || { echo "insitu rc=$?"; tail -5 $OUT/insitu.err; exit 1; }
cat $OUT/insitu.jsonl
tail -3 $OUT/insitu.err
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -5 $OUT/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print('cfg2 after', round(d['value'],3), round(d['ms_per_step'],2))"
echo done-r3ai
