#!/bin/bash
# round 3, call U: in-situ search passes at cfg2 (no-split, then isolated alternatives), chained
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r3u
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 500 python tools/insitu_tune.py --config cfg2 --top 40 --nosplit --alts-only --out $OUT/t1.json > $OUT/insitu1.jsonl 2> $OUT/insitu1.err || { echo "insitu1 rc=$?"; tail -5 $OUT/insitu1.err; exit 1; }
cat $OUT/insitu1.jsonl
T=tuning/fsmi_conv.json; [ -f $OUT/t1.json ] && T=$OUT/t1.json
FSMI_TUNE_PATH=$T timeout -k 10 900 python tools/insitu_tune.py --config cfg2 --top 30 --alts 3 --out $OUT/t2.json > $OUT/insitu2.jsonl 2> $OUT/insitu2.err || { echo "insitu2 rc=$?"; tail -5 $OUT/insitu2.err; exit 1; }
cat $OUT/insitu2.jsonl
