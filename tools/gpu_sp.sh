#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
export SP_BLOCKS=8192 SP_PER=1 SP_TILE2=1
SP_T=20 timeout -k 10 120 python tools/store_pattern.py 1,1 > $OUT/r02f_sp_T20.json 2>&1 || exit 2
SP_T=200 timeout -k 10 120 python tools/store_pattern.py 1,1 > $OUT/r02f_sp_T200.json 2>&1 || exit 2
echo done
