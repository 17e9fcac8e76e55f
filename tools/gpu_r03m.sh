#!/bin/bash
# Round-3 verification session: the whole -m gpu suite, config 4 (tools/bench_bfs.py 10^7, 10^8),
# then tools/gpu_session.sh's bench + rocprofv3 passes (K = 20 and K = 200).  Chained.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03m}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/${TAG}_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_bfs.py 10000000,100000000 > $OUT/${TAG}_bfs.json 2> $OUT/${TAG}_bfs.err || exit 2
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/${TAG}_bench_k20.json 2> $OUT/${TAG}_bench_k20.err || exit 3
bash $R/profile_cmd.sh ${TAG}_k20 --steps 20 --warmup 5 || exit 4
bash $R/profile_cmd.sh ${TAG} || exit 5
echo session-done
