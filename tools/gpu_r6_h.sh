# round-6 GPU step H: unconditional clamped loads in the window staging (dwconv, conv_1in) and the 16-wave
# Cout=1 head conv: their tests, then a same-box cfg2 A/B against the previous library (FSMI_LIB)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r6h
mkdir -p $O
timeout -k 10 400 python -u -m pytest "tests/test_gpu_backbone.py::test_dwconv_slices" "tests/test_gpu_parity.py::test_conv3x3_cout1_vs_torch" \
  "tests/test_gpu_parity.py::test_update_step_golden" "tests/test_gpu_parity.py::test_e2e_vs_reference_golden" \
  tests/test_gpu_ctx_pre.py -q -x --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || exit $?
ab() {   # ab NAME ENV...
  local name=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/ab_$name.json 2> $O/ab_$name.err || return $?
  python -c "import json; d=json.load(open('$O/ab_$name.json')); print('$name', round(d['value'], 3), 'pairs/s', round(d['ms_per_step'], 2), 'ms')" >> $O/ab.txt
}
for r in 1 2 3; do
  ab base_r$r FSMI_LIB=$GRAFT_REPO_ROOT/foundationstereo_amd/_lib/libfsmi_base.so || exit $?
  ab new_r$r || exit $?
done
cat $O/ab.txt
