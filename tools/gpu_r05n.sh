#!/bin/bash
# Round-5 session n: the sharded-BFS arena store -- its tests, the bench's search variants, and a
# rocprofv3 kernel trace of config 4's searches (per-kernel time of the sharded BFS vs the device BFS).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05n}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_sbfs.py tests/test_gpu_bfs.py tests/test_gpu_search_scale.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/${TAG}_gpu_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-step-api --no-learner --no-graph --no-desync --no-obs8 --no-config2 > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err || exit 4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_trace -o s --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu --no-step-api --no-learner --no-graph --no-desync --no-obs8 --no-config2 > $OUT/${TAG}_trace.log 2>&1 || exit 5
echo session-done
