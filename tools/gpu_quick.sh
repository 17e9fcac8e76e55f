#!/bin/bash
# Quick GPU check after a kernel change: the -m gpu suite, then bench.py at L = 36 (the driver's
# K = 20 command) and L = 128 (config 5's per-GPU shard), no CPU baseline.  Each step has its
# own time limit and the steps are chained, so a failure ends the call.
#   bash tools/gpu_quick.sh TAG [pytest -k expression]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-quick}
K=${2:-}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "$K" > $OUT/${TAG}_gpu_tests.log 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/${TAG}_gpu_tests.log 2>&1
fi
rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/${TAG}_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu > $OUT/${TAG}_bench_L36.json 2> $OUT/${TAG}_bench_L36.err || exit 3
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --L 128 --no-bfs --no-desync > $OUT/${TAG}_bench_L128.json 2> $OUT/${TAG}_bench_L128.err || exit 4
echo quick-done
