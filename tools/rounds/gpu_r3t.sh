#!/bin/bash
# round 3, call T: in-situ search of "no split-K" per shape at cfg2 (current tiles)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r3t
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 1100 python tools/insitu_tune.py --config cfg2 --top 40 --nosplit --alts-only --out $OUT/fsmi_conv.json > $OUT/insitu.jsonl 2> $OUT/insitu.err || { echo "insitu rc=$?"; tail -5 $OUT/insitu.err; exit 1; }
cat $OUT/insitu.jsonl
