#!/bin/bash
# BFS key-in-table layout (tests + A/B bench) and the headline's spread over fresh processes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03i}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_search_scale.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "device_bfs or config4" > $OUT/${TAG}_bfs_tests.log 2>&1 || { tail -5 $OUT/${TAG}_bfs_tests.log; exit 1; }
tail -2 $OUT/${TAG}_bfs_tests.log
timeout -k 10 300 python -u tools/bench_bfs.py 1e7,1e8 > $OUT/${TAG}_bfs.json 2> $OUT/${TAG}_bfs.err || exit 2
echo bfs-bench-done
for i in 1 2 3; do
  timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-step-api --no-learner --no-bfs --no-desync --no-obs8 > $OUT/${TAG}_bench_p$i.json 2> $OUT/${TAG}_bench_p$i.err || exit 3
  timeout -k 10 120 python -u tools/rollout_parts.py 36 > $OUT/${TAG}_parts_p$i.json 2> $OUT/${TAG}_parts_p$i.err || exit 4
done
echo spread-done
