#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02m}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_search_scale.py -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/${TAG}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 tools/greedy_sweep.py ${SWEEP:-32,64,128,256} > $OUT/${TAG}_sweep.json 2> $OUT/${TAG}_sweep.err || exit 3
echo done
