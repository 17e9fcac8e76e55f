#!/bin/bash
# One GPU session: the -m gpu suite, then the bench at the driver's K = 20 and at K = 200.
# Each GPU step has its own time limit; steps are chained so a failure ends the session.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/${TAG}_gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu > $OUT/${TAG}_bench_k20.json 2> $OUT/${TAG}_bench_k20.err || exit 3
timeout -k 10 300 python -u bench.py --steps 200 --warmup 10 --no-cpu --no-learner --no-graph --no-bfs > $OUT/${TAG}_bench_k200.json 2> $OUT/${TAG}_bench_k200.err || exit 4
SP_T=4 SP_B=65536 timeout -k 10 60 python tools/store_pattern.py 9,1 > $OUT/${TAG}_store_pattern_T4.json 2>&1 || exit 5
echo session-done
