#!/bin/bash
# round 3, call E: conv ablations (FSMI_CONV_DBG: 1 weights from one line, 2 no halo reloads)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r3e
rm -rf $OUT; mkdir -p $OUT
for d in 0 1 2 3; do
  FSMI_CONV_DBG=$d timeout -k 10 300 python tools/tile_ab.py --set loop --only gru04.conv1,gru04.conv0,gru04.q_l,gru04.zr_s > $OUT/dbg$d.jsonl 2> $OUT/dbg$d.err || { echo "rc=$?"; tail -3 $OUT/dbg$d.err; }
  echo "== dbg $d"; cat $OUT/dbg$d.jsonl | cut -c1-110
done
