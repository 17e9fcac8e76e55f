#!/bin/bash
# GPU session: the new/changed test files, then interleaved A/B of the rollout builds in abl/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02b}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_words.py tests/test_gpu_sbfs.py tests/test_gpu_search_scale.py -m gpu -q --maxfail=20 --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/${TAG}_gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for mode in "--T 20" "--T 200" "--T 20 --desync" "--T 200 --desync"; do
  timeout -k 10 300 python -u tools/ab_libs.py abl/old.so abl/new.so --reps 5 $mode > $OUT/${TAG}_ab_$(echo $mode | tr -d ' -').json 2>&1 || exit 3
done
echo session-done
