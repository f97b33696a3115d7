# round-6 GPU step I: hardware queues per process (GPU_MAX_HW_QUEUES, HIP default 4) for the replayed
# 4-stream step: same-box cfg2 A/B 4 / 8 / 16, and the motion path on the main stream, three alternating rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r6i
mkdir -p $O
ab() {   # ab NAME ENV...
  local name=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/ab_$name.json 2> $O/ab_$name.err || return $?
  python -c "import json; d=json.load(open('$O/ab_$name.json')); print('$name', round(d['value'], 3), 'pairs/s', round(d['ms_per_step'], 2), 'ms')" >> $O/ab.txt
}
for r in 1 2 3; do
  ab q4_r$r GPU_MAX_HW_QUEUES=4 || exit $?
  ab q8_r$r GPU_MAX_HW_QUEUES=8 || exit $?
  ab q16_r$r GPU_MAX_HW_QUEUES=16 || exit $?
  ab motion_main_r$r FSMI_MOTION_ON_MAIN=1 || exit $?
done
cat $O/ab.txt
