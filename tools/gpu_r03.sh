#!/bin/bash
# Round-3 GPU session after a kernel change: the step/rollout/learner/parity GPU tests, the
# driver's bench command at L = 36 and L = 128 (no CPU baseline), the rollout SQ counters and the
# move microbenchmark.  Each GPU step under its own time limit, chained.
#   bash tools/gpu_r03.sh TAG [pytest -k expression]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03}
K=${2:-"rollout or error or in_place or step or learner or parity or words or features or canonicalize or bad_parents"}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 800 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 300 --timeout-method thread -p no:cacheprovider -k "$K" > $OUT/${TAG}_gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 $OUT/${TAG}_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-bfs > $OUT/${TAG}_bench_L36.json 2> $OUT/${TAG}_bench_L36.err || exit 3
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --L 128 --no-bfs --no-desync > $OUT/${TAG}_bench_L128.json 2> $OUT/${TAG}_bench_L128.err || exit 4
timeout -k 10 120 python -u tools/move_probe.py > $OUT/${TAG}_move_probe.json 2>&1 || exit 5
bash tools/profile_rollout_sq.sh $TAG > $OUT/${TAG}_rsq.log 2>&1 || exit 6
echo r03-session-done
