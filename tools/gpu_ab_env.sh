#!/bin/bash
# A/B of environment settings on the default bench, interleaved: ENVS="A=1,B=2 C=3 ..." (, joins; "-" = none)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-abenv}; mkdir -p $OUT
for i in $(seq 1 ${ROUNDS:-2}); do
  for e in $ENVS; do
    ev=""; [ "$e" != "-" ] && ev=$(echo "$e" | tr ',' ' ')
    env $ev timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 $BENCH_ARGS > $OUT/b_$i.json 2>>$OUT/b.err || { echo "bench $e rc=$?"; tail -5 $OUT/b.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/b_$i.json')); print('$e', $i, round(d['value'],3), round(d['ms_per_step'],2), 'conv', round(d['roofline_conv']['total_ms'],2), 'ovf', d.get('range_overflow'))"
  done
done
