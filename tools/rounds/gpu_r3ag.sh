#!/bin/bash
# round 3, call AG: pipelined tiles with a rolling single-buffer B prefetch (FSMI_PIPE_ROLLB=1) vs the
# double-buffered B fragments (libfsmi_rb0.so): pipe tests, loop-layer tile A/B, cfg2 bench A/B

set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r3ag
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipe.py -m gpu -x -q --timeout 250 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for lib in libfsmi.so libfsmi_rb0.so; do
FSMI_LIB=foundationstereo_amd/_lib/$lib timeout -k 10 300 python tools/tile_ab.py --set loop > $OUT/loop_$lib.jsonl 2> $OUT/loop_$lib.err || { echo "loop rc=$?"; tail -5 $OUT/loop_$lib.err; exit 1; }
done
python - <<'P'
import json
def load(f):
    return {(d['layer'], d['cfg'], d['nsplit']): d for d in map(json.loads, open(f)) if 'us' in d}
a = load('gpurun_out/r3ag/loop_libfsmi.so.jsonl'); b = load('gpurun_out/r3ag/loop_libfsmi_rb0.so.jsonl')
for k in a:
    if k in b: print(k, 'rb1', a[k]['us'], 'rb0', b[k]['us'], 'err', a[k].get('rel_err'))
P
for lib in libfsmi.so libfsmi_rb0.so libfsmi.so libfsmi_rb0.so; do
FSMI_LIB=foundationstereo_amd/_lib/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $OUT/bench_$lib.json 2> $OUT/bench_$lib.err || { echo "bench rc=$?"; tail -5 $OUT/bench_$lib.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench_$lib.json').read().strip().splitlines()[-1]); print('$lib', round(d['value'],3), round(d['ms_per_step'],2), round(d['roofline_conv']['frac'],4), round(d['roofline_conv_step']['frac'],4))"
done
echo done-r3ag
