# round-6 final GPU check A: full -m gpu suite, smoke, then the cfg2 round profile (bench line, rocprof
# kernel-trace stats of the same command, FETCH_SIZE / WRITE_SIZE PMC passes; tools/gpu_round_profile.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r6final
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; echo "gpu tests rc=$rc" >> $O/gpu_tests.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.txt 2>&1 || exit $?
CONFIG=cfg2 timeout -k 10 900 bash tools/gpu_round_profile.sh > $O/profile_cfg2.log 2>&1
