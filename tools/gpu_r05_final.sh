#!/bin/bash
# Round-5 verification of the committed tree: the whole -m gpu suite, __graft_entry__.smoke(), the
# driver's bench command (CPU baseline included), config 5's line, config 4's BFS sweep.  Each
# step under its own limit, chained.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05final}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
rocm-smi --showmemvendor --showvbios --showclkfrq --showperflevel > $OUT/${TAG}_box.txt 2>&1 || true
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/${TAG}_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke-ok')" > $OUT/${TAG}_smoke.log 2>&1 || exit 2
tail -2 $OUT/${TAG}_smoke.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err || exit 3
timeout -k 10 400 python -u bench.py --workload step --L 128 --no-cpu --no-bfs --no-search > $OUT/${TAG}_config5.json 2> $OUT/${TAG}_config5.err || exit 4
echo final-done
