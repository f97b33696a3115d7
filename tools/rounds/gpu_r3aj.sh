#!/bin/bash
# round 3, call AJ: fast-precision range recovery check (two fast bench runs, one with the lookup at
# 4 channels per wave), then the in-situ re-tune of call AI
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r3aj
rm -rf $OUT; mkdir -p $OUT
for r in 1 2; do
timeout -k 10 300 python bench.py --precision fast --no-cpu-baseline --steps 20 > $OUT/fast$r.json 2> $OUT/fast$r.err || { echo "fast rc=$?"; tail -5 $OUT/fast$r.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/fast$r.json').read().strip().splitlines()[-1]); print('fast', d['value'], d['range_overflow'], d['range_recoveries'])"
done
bash tools/rounds/gpu_r3ai.sh || exit 1
echo done-r3aj
