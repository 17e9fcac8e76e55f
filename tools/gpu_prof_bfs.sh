#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_bfs_${1:-r02h}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o bfs --output-format csv -- python3 $R/tools/bench_bfs.py 1e7 > $OUT/trace.log 2>&1 || exit 2
echo done
