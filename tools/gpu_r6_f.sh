# round-6 GPU check F (HEAD after the context-part hoist): full -m gpu suite, smoke, the cfg2 headline bench,
# a rocprof kernel trace of the headline bench command and the replay timeline (each step time-limited)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r6f
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; echo "gpu tests rc=$rc" >> $O/gpu_tests.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $O/cfg2_bench.json 2> $O/cfg2_bench.err || exit $?
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o cfg2 -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/cfg2_under_rocprof.json 2> $GRAFT_REPO_ROOT/$O/cfg2_under_rocprof.err
rc=$?; echo "rocprof rc=$rc" >> $GRAFT_REPO_ROOT/$O/cfg2_under_rocprof.err
[ $rc -eq 0 ] || exit $rc
cd $GRAFT_REPO_ROOT && timeout -k 10 300 python -u tools/replay_timeline.py --out $O/replay_timeline.txt > $O/replay_timeline.log 2>&1
