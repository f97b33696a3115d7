#!/bin/bash
# round 3, call AL: split-K off for the small GRU levels (FSMI_SPLIT_MAXPIX: 2D maps of at most N
# pixels run unsplit) -- end-to-end A/B, two runs each, alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r3al
rm -rf $OUT; mkdir -p $OUT
for r in 1 2; do
for mp in 0 1200 4800; do
FSMI_SPLIT_MAXPIX=$mp timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $OUT/b_${mp}_$r.json 2> $OUT/b_${mp}_$r.err || { echo "bench rc=$?"; tail -5 $OUT/b_${mp}_$r.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/b_${mp}_$r.json').read().strip().splitlines()[-1]); print('maxpix $mp run $r', round(d['value'],3), round(d['ms_per_step'],2))"
done
done
echo done-r3al
