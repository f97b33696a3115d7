set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_backbone.py -v --timeout 400 --timeout-method thread > gpurun_out/r6_backbone_tests.txt 2>&1
rc=$?
echo "backbone tests rc=$rc" >> gpurun_out/r6_backbone_tests.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/r6_smoke.txt 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --with-backbone --steps 5 --warmup 2 > gpurun_out/r6_cfg2_backbone_bench.json 2> gpurun_out/r6_cfg2_backbone_bench.err
