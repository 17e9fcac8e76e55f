#!/bin/bash
# after a device-BFS change: the BFS / search GPU tests, then tools/bench_bfs.py at 10^7 and 10^8
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
TAG=${1:-bfs}
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -k "bfs or search or sbfs" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_bfs.py 10000000,100000000 > gpurun_out/${TAG}_bfs.json 2> gpurun_out/${TAG}_bfs.err || exit 2
echo bfs-check-done
