# round-6 GPU check A: full -m gpu suite, smoke, the cfg2 headline and --with-backbone benches, and the
# dependency-based replay timeline (each step time-limited; stops at the first failure)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r6a
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; echo "gpu tests rc=$rc" >> $O/gpu_tests.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $O/cfg2_bench.json 2> $O/cfg2_bench.err || exit $?
timeout -k 10 400 python -u bench.py --with-backbone > $O/cfg2_bb_bench.json 2> $O/cfg2_bb_bench.err || exit $?
timeout -k 10 300 python -u tools/replay_timeline.py --out $O/replay_timeline.txt > $O/replay_timeline.log 2>&1
