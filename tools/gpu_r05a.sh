#!/bin/bash
# Round-5 session a: the -m gpu suite, the small-batch step A/B (config 2's B = 65,536), the
# driver's bench command and config 5's line.  Each GPU step under its own limit; a crash
# (status other than 0 / 1 from pytest) ends the call.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05a}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
rocm-smi --showmemvendor --showvbios > $OUT/${TAG}_box.txt 2>&1 || true
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/${TAG}_gpu_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/ab_step.py ab5/libacx_nosmall.so ab5/libacx_small.so ab5/libacx_small9.so --L 36 --B 65536 --K 200 --reps 7 > $OUT/${TAG}_ab_small.json 2> $OUT/${TAG}_ab_small.err || exit 3
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err || exit 4
timeout -k 10 400 python -u bench.py --workload step --L 128 --no-cpu --no-bfs --no-search > $OUT/${TAG}_config5.json 2> $OUT/${TAG}_config5.err || exit 5
echo session-done
