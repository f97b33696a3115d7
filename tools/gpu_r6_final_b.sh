# round-6 final GPU check B: cfg3 (per-GPU share, 4 pairs) and cfg5 (hierarchical) bench lines with their
# rocprof stats (no PMC), the cfg2 --with-backbone line, and the cfg2 replay timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r6final
mkdir -p $O
CONFIG=cfg3 PPG=4 NO_PMC=1 STEPS=3 timeout -k 10 500 bash tools/gpu_round_profile.sh > $O/profile_cfg3.log 2>&1 || exit $?
CONFIG=cfg5 NO_PMC=1 STEPS=3 timeout -k 10 500 bash tools/gpu_round_profile.sh > $O/profile_cfg5.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --with-backbone > $O/cfg2_bb_bench.json 2> $O/cfg2_bb_bench.err || exit $?
timeout -k 10 300 python -u tools/replay_timeline.py --out $O/replay_timeline.txt > $O/replay_timeline.log 2>&1
