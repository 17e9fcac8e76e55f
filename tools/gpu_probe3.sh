#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 300 python3 tools/placement_patterns.py 6 > $OUT/r02y_patterns.json 2> $OUT/r02y_patterns.err || exit 2
timeout -k 10 300 python3 tools/greedy_sweep.py 64 > $OUT/r02y_sweep.json 2> $OUT/r02y_sweep.err || exit 3
echo done
