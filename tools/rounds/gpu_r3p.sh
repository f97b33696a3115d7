#!/bin/bash
# round 3, call P: B prefetch in the register-weight (wreg) tiles, same-box A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r3p
rm -rf $OUT; mkdir -p $OUT
for i in 1 2 3; do
for v in "" _nobpref; do
FSMI_LIB=foundationstereo_amd/_lib/libfsmi$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $OUT/bench${v}_${i}.json 2> $OUT/bench${v}_${i}.err || { echo "bench rc=$?"; tail -5 $OUT/bench${v}_${i}.err; exit 1; }
done
done
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r3p/bench*.json")):
    d=json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"],3), round(d["ms_per_step"],2), round(d["roofline"]["frac"],3), round(d["roofline_conv"]["frac"],3))
PY
