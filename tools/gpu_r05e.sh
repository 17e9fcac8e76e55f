#!/bin/bash
# Round-5 session e: a -m gpu subset, the default bench line (no CPU baseline), then config 2's
# probe (tools/config2_probe.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05e}
K=${2:-learner}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "$K" > $OUT/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/${TAG}_gpu_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err || exit 4
timeout -k 10 300 python -u tools/config2_probe.py ab5/libacx_small.so ab5/libacx_small_ntsc.so ab5/libacx_nosmall.so --K 100 --reps 3 > $OUT/${TAG}_config2_probe.json 2> $OUT/${TAG}_config2_probe.err || exit 3
echo session-done
