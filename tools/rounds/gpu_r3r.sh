#!/bin/bash
# round 3, call R: in-situ (end-to-end) tile / split search over the round-3 tiles at cfg2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r3r
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 1100 python tools/insitu_tune.py --config cfg2 --top 28 --alts 3 --out $OUT/fsmi_conv.json > $OUT/insitu.jsonl 2> $OUT/insitu.err || { echo "insitu rc=$?"; tail -5 $OUT/insitu.err; exit 1; }
tail -3 $OUT/insitu.jsonl
