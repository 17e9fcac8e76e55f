#!/bin/bash
# Round-5 session q: after a step-kernel change -- the whole -m gpu suite, the learner probe
# (tools/learner_probe.py) and the bench (no CPU baseline, no searches).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05q}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/${TAG}_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/learner_probe.py > $OUT/${TAG}_learner_probe.json 2> $OUT/${TAG}_learner_probe.err || exit 3
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-bfs --no-search > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err || exit 4
echo session-done
