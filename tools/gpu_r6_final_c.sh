# round-6 closing GPU check at HEAD: full -m gpu suite, smoke, the cfg2 headline bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r6close
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; echo "gpu tests rc=$rc" >> $O/gpu_tests.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $O/cfg2_bench.json 2> $O/cfg2_bench.err
