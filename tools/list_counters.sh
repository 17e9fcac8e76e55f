#!/bin/bash
# rocprofv3's counter list on the box (names, blocks, dimensions), for choosing PMC passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/counters
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/list.txt 2>&1 || timeout -k 10 120 rocprofv3 --list-avail > $OUT/list.txt 2>&1
grep -c . $OUT/list.txt
