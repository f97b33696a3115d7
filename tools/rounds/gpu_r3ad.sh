#!/bin/bash
# round 3, call AD: per-block timelines of the big loop convs (plain register tiles, which carry the
# debug stamps), parity vs fast builds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r3ad
rm -rf $OUT; mkdir -p $OUT
for prec in parity fast; do
for spec in "gru04.conv1 9 4" "gru04.conv1 9 1" "gru04.conv0 8 1" "gru04.zr_l 9 3" "enc.convc2 9 1"; do
set -- $spec
echo "== $prec $spec"
FSMI_PRECISION=$prec timeout -k 10 120 python tools/conv_phases.py --layer $1 --cfg $2 --nsplit $3 > $OUT/ph_${prec}_$1_$2_$3.txt 2>&1 || { echo "rc=$?"; tail -5 $OUT/ph_${prec}_$1_$2_$3.txt; exit 1; }
grep -v amdgpu.ids $OUT/ph_${prec}_$1_$2_$3.txt
done
done
echo done-r3ad
