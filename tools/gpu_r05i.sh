#!/bin/bash
# Round-5 session i: the dual-tile rollout A/B (tools/ab_rollout.py, same buffers, trajectories
# compared) and config 5's line with the current library.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05i}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u tools/ab_rollout.py ab5/libacx_roll1.so ab5/libacx_roll2.so --K 20,200 --reps 5 > $OUT/${TAG}_ab_dual.json 2> $OUT/${TAG}_ab_dual.err || exit 1
timeout -k 10 500 python -u bench.py --workload step --L 128 --no-cpu --no-bfs --no-search > $OUT/${TAG}_config5.json 2> $OUT/${TAG}_config5.err || exit 2
echo session-done
