#!/bin/bash
# round 3, call C: depth-tile + range tests, e2e parity, depth tile A/B bench, kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r3c
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_depth.py tests/test_gpu_range.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; grep -v MIOpen $OUT/tests.log | tail -40; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "e2e or conv3d or hourglass" --timeout 600 --timeout-method thread > $OUT/tests2.log 2>&1 || { echo "tests2 rc=$?"; grep -v MIOpen $OUT/tests2.log | tail -40; exit 1; }
tail -2 $OUT/tests2.log
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $OUT/bench_depth_$i.json 2> $OUT/bench_depth_$i.err || { echo "bench rc=$?"; tail -5 $OUT/bench_depth_$i.err; exit 1; }
FSMI_DEPTH_TILE=0 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $OUT/bench_nodepth_$i.json 2> $OUT/bench_nodepth_$i.err || { echo "bench rc=$?"; tail -5 $OUT/bench_nodepth_$i.err; exit 1; }
done
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r3c/bench_*.json")):
    d=json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"],3), round(d["ms_per_step"],2), round(d["roofline"]["frac"],3), round(d["roofline_conv"]["frac"],3), d.get("range_overflow"))
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $OUT/trace_bench.json 2> $OUT/trace.err || { echo "trace rc=$?"; tail -5 $OUT/trace.err; exit 1; }
find $OUT/trace -name "*kernel_stats.csv" -exec head -30 {} \; | cut -c1-200
