#!/bin/bash
# Round-5 session f: learner tests + bench (no CPU baseline), then rocprofv3 over config 2's step
# launch (kernel trace + one SQ counter pass).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05f}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -k learner > $OUT/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/${TAG}_gpu_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-bfs --no-search > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err || exit 4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_c2trace -o c2 --output-format csv -- python3 $R/tools/step_pmc.py --L 36 --B 65536 --K 50 > $OUT/${TAG}_c2trace.log 2>&1 || exit 5
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU -d $OUT/${TAG}_c2pmc -o c2 --output-format csv -- python3 $R/tools/step_pmc.py --L 36 --B 65536 --K 50 > $OUT/${TAG}_c2pmc.log 2>&1 || exit 6
echo session-done
