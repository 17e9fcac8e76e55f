#!/bin/bash
# One profiling session (round 4): rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes
# (profile_cmd.sh) of
#   TAG_k20      the driver's command (bench.py --steps 20 --warmup 5), headline rollout
#   TAG_step128  config 5's kernel: bench.py --workload step --L 128 (in-place acx_step)
#   TAG_step36   the same at L = 36
# then bench.py --workload step --L 128 on its own (the config-5 per-GPU line), and a kernel +
# memory-copy trace of the device BFS to 10^7 nodes (tools/bench_bfs.py): the log must show no
# copy whose completion never arrived.  Each step under its own limit, chained.
#   bash tools/gpu_profile_session.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
NOV="--no-search --no-bfs"
bash profile_cmd.sh ${TAG}_k20 --steps 20 --warmup 5 $NOV || exit 1
bash profile_cmd.sh ${TAG}_step128 --workload step --L 128 --steps 20 --warmup 3 $NOV --no-learner --no-graph || exit 2
bash profile_cmd.sh ${TAG}_step36 --workload step --L 36 --steps 20 --warmup 3 $NOV --no-learner --no-graph || exit 3
cd $R
timeout -k 10 300 python -u bench.py --workload step --L 128 --steps 50 --warmup 5 --no-search --no-bfs > $OUT/${TAG}_bench_step128.json 2> $OUT/${TAG}_bench_step128.err || exit 4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $OUT/${TAG}_bfs_trace -o bfs --output-format csv -- python3 $R/tools/bench_bfs.py 10000000 > $OUT/${TAG}_bfs_trace.log 2>&1 || exit 5
echo session-done
