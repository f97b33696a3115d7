#!/bin/bash
# round 3, call AF: per-block timelines of gru04.conv1 (cfg 9, split 4) under the conv ablations
# (FSMI_CONV_DBG 1: every tap's weights from one line, 2: no halo reloads, 3: both)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r3af
rm -rf $OUT; mkdir -p $OUT
for d in 0 1 2 3; do
for spec in "gru04.conv1 9 4" "gru04.conv0 8 1"; do
set -- $spec
echo "== dbg $d $spec"
FSMI_CONV_DBG=$d timeout -k 10 120 python tools/conv_phases.py --layer $1 --cfg $2 --nsplit $3 > $OUT/ph_d${d}_$1.txt 2>&1 || { echo "rc=$?"; tail -5 $OUT/ph_d${d}_$1.txt; exit 1; }
grep -v amdgpu.ids $OUT/ph_d${d}_$1.txt
done
done
echo done-r3af
