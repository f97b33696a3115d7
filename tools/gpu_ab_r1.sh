#!/bin/bash
# A/B against the round-1 tree (ab_r1/, git-ignored copy of commit 49eee76 with its own build) on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=$PWD/gpurun_out/${TAG:-abr1}; mkdir -p $OUT
for i in $(seq 1 ${ROUNDS:-2}); do
  (cd ab_r1 && timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 > $OUT/r1_$i.json 2>>$OUT/b.err) || { echo "r1 rc=$?"; tail -5 $OUT/b.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/r1_$i.json')); print('r1', $i, round(d['value'],3), round(d['ms_per_step'],2), 'conv', round(d['roofline_conv']['total_ms'],2))"
  for v in $LIBS; do
    if [ "$v" = "default" ]; then L=foundationstereo_amd/_lib/libfsmi.so; else L=foundationstereo_amd/_lib/libfsmi_$v.so; fi
    FSMI_LIB=$L timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 $BENCH_ARGS > $OUT/b_${v}_$i.json 2>>$OUT/b.err || { echo "bench $v rc=$?"; tail -5 $OUT/b.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/b_${v}_$i.json')); print('$v', $i, round(d['value'],3), round(d['ms_per_step'],2), 'conv', round(d['roofline_conv']['total_ms'],2))"
  done
done
