#!/bin/bash
# round 3, call Z: lookup channels-per-wave A/B in the bench (FSMI_LOOKUP_CPC 2 / 4 / 7 builds),
# SQ counters (MFMA busy, instruction mix) for the geometry kernels (all-pairs correlation MFMA,
# build, lookup), rocprof kernel stats of the fast-precision bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r3z
rm -rf $OUT; mkdir -p $OUT
for lib in libfsmi.so libfsmi_cpc2.so libfsmi_cpc7.so libfsmi.so; do
FSMI_LIB=foundationstereo_amd/_lib/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $OUT/bench_$lib.json 2> $OUT/bench_$lib.err || { echo "bench rc=$?"; tail -5 $OUT/bench_$lib.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench_$lib.json').read().strip().splitlines()[-1]); print('$lib', round(d['value'],3), round(d['ms_per_step'],2), round(d['roofline']['frac'],4), round(d['roofline']['avg_us'],2))"
done
P1="SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-include-regex 'allpairs|normalize_cols|build_stem|geo_lookup|volume_pyramid' --output-format csv -d $OUT/pmc_P$i -o pmc -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/pmc_P$i.json 2> $OUT/pmc_P$i.err || { echo "pmc P$i rc=$?"; tail -5 $OUT/pmc_P$i.err; exit 1; }
done
python3 tools/conv_pmc_summary.py $OUT --top 8 --out $OUT/sq_geometry_cfg2.json > $OUT/sq_geometry_table.txt
cat $OUT/sq_geometry_table.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_fast -o run -- python3 bench.py --precision fast --no-cpu-baseline > $OUT/trace_fast_bench.json 2> $OUT/trace_fast.err || { echo "trace rc=$?"; tail -5 $OUT/trace_fast.err; exit 1; }
cat $OUT/trace_fast_bench.json
echo done-r3z
