# round-6 GPU check: full -m gpu suite, smoke, the cfg2 headline bench, a rocprof kernel trace of the
# --with-backbone step and the census of torch convs left in the forward (each step time-limited)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r6s
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; echo "gpu tests rc=$rc" >> $O/gpu_tests.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $O/cfg2_bench.json 2> $O/cfg2_bench.err || exit $?
timeout -k 10 200 python -u tools/torch_conv_census.py --out $O/torch_conv_census.txt > /dev/null 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_bb -o bb -- python3 $GRAFT_REPO_ROOT/bench.py --with-backbone --steps 3 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/bb_under_rocprof.json 2> $GRAFT_REPO_ROOT/$O/bb_under_rocprof.err
rc=$?; echo "rocprof bb rc=$rc" >> $GRAFT_REPO_ROOT/$O/bb_under_rocprof.err
[ $rc -eq 0 ] || exit $rc
cd $GRAFT_REPO_ROOT && timeout -k 10 300 python -u tools/replay_timeline.py --out $O/replay_timeline.txt > $O/replay_timeline.log 2>&1
