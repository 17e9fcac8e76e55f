#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02c}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
for mode in "--T 20" "--T 20 --desync" "--T 200 --desync"; do
  timeout -k 10 300 python -u tools/ab_libs.py abl/old.so abl/new.so abl/new2.so --reps 5 $mode > $OUT/${TAG}_ab_$(echo $mode | tr -d ' -').json 2>&1 || exit 3
done
for T in 1 2 5 10 20 50 100; do
  timeout -k 10 300 python -u tools/ab_libs.py abl/new2.so --reps 5 --T $T > $OUT/${TAG}_curve_T$T.json 2>&1 || exit 4
  timeout -k 10 300 python -u tools/ab_libs.py abl/new2.so --reps 5 --T $T --unpacked > $OUT/${TAG}_curveU_T$T.json 2>&1 || exit 4
done
echo session-done
