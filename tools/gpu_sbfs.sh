#!/bin/bash
# the BFS / sharded-BFS GPU tests, the one-rank sharded BFS next to the device BFS, and a
# rocprofv3 kernel trace of the latter
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02}
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_sbfs.py tests/test_gpu_search_scale.py tests/test_gpu_bfs.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 tools/bench_sbfs.py 1e6 1e7 1e8 > gpurun_out/${TAG}_sbfs.json 2> gpurun_out/${TAG}_sbfs.err || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_sbfs_${TAG} -o sbfs --output-format csv -- python3 $R/tools/bench_sbfs.py 1e7 > $R/gpurun_out/prof_sbfs_${TAG}.log 2>&1 || exit 4
echo done
