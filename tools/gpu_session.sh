#!/bin/bash
# One GPU session: the -m gpu suite, the driver's bench command, then rocprofv3 passes over the
# driver's command (K = 20) and the K = 200 default.  Each GPU step has its own time limit;
# steps are chained so a failure ends the session.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02}  # usage: bash tools/gpu_session.sh TAG  (PROFILE=0: skip the rocprofv3 passes)
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
# the box: HBM vendor, VBIOS, partition modes, clock levels (read only; the fast/slow rollout split is per box)
rocm-smi --showmemvendor --showvbios --showmemorypartition --showcomputepartition --showclkfrq --showperflevel > $OUT/${TAG}_box.txt 2>&1 || true
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/${TAG}_gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/${TAG}_gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/${TAG}_bench_k20.json 2> $OUT/${TAG}_bench_k20.err || exit 3
echo bench-done
[ "${PROFILE:-1}" = "1" ] || exit 0
bash $R/profile_cmd.sh ${TAG}_k20 --steps 20 --warmup 5 || exit 4
bash $R/profile_cmd.sh ${TAG} || exit 5
echo session-done
