#!/bin/bash
# A/B of library variants (FSMI_LIB) on the default bench, interleaved: LIBS="name1 name2 ..." ("" = default lib)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-ablibs}; mkdir -p $OUT
for i in $(seq 1 ${ROUNDS:-2}); do
  for v in $LIBS; do
    if [ "$v" = "default" ]; then L=foundationstereo_amd/_lib/libfsmi.so; else L=foundationstereo_amd/_lib/libfsmi_$v.so; fi
    FSMI_LIB=$L timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 $BENCH_ARGS > $OUT/b_${v}_$i.json 2>>$OUT/b.err || { echo "bench $v rc=$?"; tail -5 $OUT/b.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/b_${v}_$i.json')); print('$v', $i, round(d['value'],3), round(d['ms_per_step'],2), 'conv', round(d['roofline_conv']['total_ms'],2), 'ms', round(d['roofline_conv']['frac'],3), 'lookup', round(d['roofline']['avg_us'],2), round(d['roofline']['frac'],3))"
  done
done
