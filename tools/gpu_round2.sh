#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02g}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 tools/bench_bfs.py 1e7,1e8 > $OUT/${TAG}_bench_bfs.json 2> $OUT/${TAG}_bench_bfs.err || exit 3
echo session-done
