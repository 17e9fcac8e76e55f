#!/bin/bash
# rocprofv3 kernel trace of the config-4 search bench (device BFS + host-dedup BFS + expand12)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
OUT=$R/gpurun_out/prof_search_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o search --output-format csv -- python3 $R/tools/bench_search.py > $OUT/search.log 2>&1 || exit 1
echo profile-search-done
# owner-partitioned BFS (one rank) next to the device BFS: tools/bench_sbfs.py
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_sbfs -o sbfs --output-format csv -- python3 $R/tools/bench_sbfs.py 1e7 > $OUT/sbfs.log 2>&1 || exit 2
echo profile-sbfs-done
