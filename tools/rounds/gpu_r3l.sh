#!/bin/bash
# round 3, call L: A/B of the pipelined 3x3 tiles (table entries c -> 32 + c) end to end
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r3l
rm -rf $OUT; mkdir -p $OUT
for i in 1 2 3; do
FSMI_TUNE_PATH=tuning/ab/fsmi_conv_pipe.json timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $OUT/bench_pipe_$i.json 2> $OUT/bench_pipe_$i.err || { echo "bench rc=$?"; tail -5 $OUT/bench_pipe_$i.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $OUT/bench_base_$i.json 2> $OUT/bench_base_$i.err || { echo "bench rc=$?"; tail -5 $OUT/bench_base_$i.err; exit 1; }
done
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r3l/bench_*.json")):
    d=json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"],3), round(d["ms_per_step"],2), round(d["roofline"]["frac"],3), round(d["roofline_conv"]["frac"],3))
PY
