#!/bin/bash
# round 3, call V: volume conv tiles, with and without halo reloads (FSMI_CONV_DBG=2 ablation)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r3v
rm -rf $OUT; mkdir -p $OUT
for d in 0 2; do
FSMI_CONV_DBG=$d timeout -k 10 300 python tools/tile_ab.py --set vol > $OUT/vol_dbg$d.jsonl 2> $OUT/vol_dbg$d.err || { echo "rc=$?"; tail -3 $OUT/vol_dbg$d.err; exit 1; }
echo "== dbg $d"; python -c "
import json
for l in open('$OUT/vol_dbg$d.jsonl'):
    d=json.loads(l); print('  ', d['layer'], d['cfg'], d['nsplit'], d['us'], d['TF'])"
done
