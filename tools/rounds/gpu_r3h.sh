#!/bin/bash
# round 3, call H: pointwise tile with one barrier per chunk vs two (FSMI_LIB A/B)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r3h
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_range.py -m gpu -x -q -k "pw or range or safe or zero" --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; grep -v MIOpen $OUT/tests.log | tail -30; exit 1; }
tail -1 $OUT/tests.log
for v in "" _pw2bar; do
FSMI_LIB=foundationstereo_amd/_lib/libfsmi$v.so timeout -k 10 300 python tools/tile_ab.py --set loop --only gru04.zr_s,gru04.q_s,enc.convc1,head.pw1,head.pw2 > $OUT/ab$v.jsonl 2> $OUT/ab$v.err || { echo "ab rc=$?"; tail -3 $OUT/ab$v.err; exit 1; }
done
for i in 1 2; do
for v in "" _pw2bar; do
FSMI_LIB=foundationstereo_amd/_lib/libfsmi$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $OUT/bench${v}_${i}.json 2> $OUT/bench${v}_${i}.err || { echo "bench rc=$?"; tail -5 $OUT/bench${v}_${i}.err; exit 1; }
done
done
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r3h/ab*.jsonl")):
    print("==", f)
    for l in open(f):
        d=json.loads(l); print("  ", d["layer"], d["cfg"], d["nsplit"], d["us"], d["TF"])
for f in sorted(glob.glob("gpurun_out/r3h/bench*.json")):
    d=json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"],3), round(d["ms_per_step"],2), round(d["roofline_conv"]["frac"],3))
PY
