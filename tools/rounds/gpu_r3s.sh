#!/bin/bash
# round 3, call S: split-K cap A/B (auto-chosen entries; in-situ entries keep their split)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r3s
rm -rf $OUT; mkdir -p $OUT
for i in 1 2; do
for c in 2 1 3; do
FSMI_SPLIT_CAP=$c timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $OUT/bench_cap${c}_$i.json 2> $OUT/bench_cap${c}_$i.err || { echo "bench rc=$?"; tail -5 $OUT/bench_cap${c}_$i.err; exit 1; }
done
done
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r3s/bench_*.json")):
    d=json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"],3), round(d["ms_per_step"],2), round(d["roofline"]["frac"],3), round(d["roofline_conv"]["frac"],3))
PY
