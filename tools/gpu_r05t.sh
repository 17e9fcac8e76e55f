#!/bin/bash
# Round-5 session t: learner probe + bench (no CPU baseline, no searches) -- no test suite
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05t}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u tools/learner_probe.py > $OUT/${TAG}_learner_probe.json 2> $OUT/${TAG}_learner_probe.err || exit 3
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-bfs --no-search > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err || exit 4
echo session-done
