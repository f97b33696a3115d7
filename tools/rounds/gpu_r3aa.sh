#!/bin/bash
# round 3, call AA: pipelined (one barrier per plane) depth-blocked (17,1,1) conv -- parity tests,
# tile A/B against the two-barrier walk (libfsmi_dp0.so), cfg2 bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r3aa
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_depth.py -m gpu -x -q --timeout 250 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for lib in libfsmi.so libfsmi_dp0.so; do
FSMI_LIB=foundationstereo_amd/_lib/$lib timeout -k 10 200 python tools/tile_ab.py --set depth > $OUT/depth_$lib.jsonl 2> $OUT/depth_$lib.err || { echo "depth rc=$?"; tail -5 $OUT/depth_$lib.err; exit 1; }
echo "== $lib"; python -c "
import json
for l in open('$OUT/depth_$lib.jsonl'):
    d=json.loads(l)
    if d.get('cfg') == 30: print('  ', d['layer'], d['cfg'], d.get('us'), d.get('TF'), d.get('rel_err'))"
done
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -5 $OUT/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print('cfg2', round(d['value'],3), round(d['ms_per_step'],2))"
echo done-r3aa
