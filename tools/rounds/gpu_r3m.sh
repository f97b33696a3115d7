#!/bin/bash
# round 3, call M: B fragments read one step ahead in the pipelined tiles
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r3m
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipe.py tests/test_gpu_parity.py -m gpu -x -q -k "pipe or e2e" --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; grep -v MIOpen $OUT/tests.log | tail -30; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 600 python tools/tile_ab.py --set loop --only gru04.conv0,gru04.conv1,gru04.zr_l,gru04.q_l,enc.convc2,enc.conv,gru08.conv1,gru08.conv0 > $OUT/tile_ab.jsonl 2> $OUT/tile_ab.err || { echo "tile_ab rc=$?"; tail -3 $OUT/tile_ab.err; exit 1; }
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $OUT/bench_$i.json 2> $OUT/bench_$i.err || { echo "bench rc=$?"; tail -5 $OUT/bench_$i.err; exit 1; }
done
python - <<'PY'
import json,glob
for l in open("gpurun_out/r3m/tile_ab.jsonl"):
    d=json.loads(l); print("  ", d["layer"], d["cfg"], d["nsplit"], d["us"], d["TF"])
for f in sorted(glob.glob("gpurun_out/r3m/bench_*.json")):
    d=json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"],3), round(d["ms_per_step"],2), round(d["roofline"]["frac"],3), round(d["roofline_conv"]["frac"],3))
PY
