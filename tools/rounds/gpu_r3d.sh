#!/bin/bash
# round 3, call D: depth-tile + pipelined-tile tests, per-layer tile A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r3d
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_depth.py tests/test_gpu_pipe.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; grep -v MIOpen $OUT/tests.log | tail -40; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 600 python tools/tile_ab.py --set all > $OUT/tile_ab.jsonl 2> $OUT/tile_ab.err || { echo "tile_ab rc=$?"; tail -5 $OUT/tile_ab.err; exit 1; }
cat $OUT/tile_ab.jsonl
