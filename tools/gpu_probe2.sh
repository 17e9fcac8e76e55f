#!/bin/bash
# placement probe (fresh vs kept allocations at T_buf 20 / 200), then the BFS profile passes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 300 python3 tools/placement_probe.py 20 20,200 4 free > $OUT/r02q_place_free.json 2> $OUT/r02q_place_free.err || exit 2
timeout -k 10 300 python3 tools/placement_probe.py 20 20,200 3 keep > $OUT/r02q_place_keep.json 2> $OUT/r02q_place_keep.err || exit 3
bash tools/profile_bfs.sh r02q || exit 4
echo done
