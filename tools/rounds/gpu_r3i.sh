#!/bin/bash
# round 3, call I: per-block phase timelines of the big loop convs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for L in "gru04.conv1 --cfg 9 --nsplit 2" "gru04.conv1 --cfg 9 --nsplit 1" "gru04.conv0 --cfg 8 --nsplit 1" "gru04.zr_s --cfg 4 --nsplit 2" "gru04.zr_s --cfg 4 --nsplit 1" "enc.convc2 --cfg 9 --nsplit 2"; do
  timeout -k 10 120 python tools/conv_phases.py --layer $L 2>&1 | grep -v MIOpen || exit 1
done
