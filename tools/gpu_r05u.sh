#!/bin/bash
# Round-5 session u: after a step-kernel change -- the whole -m gpu suite, the learner probe and
# a kernel trace of it (per-kernel split of the four-launch path)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05u}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/${TAG}_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/learner_probe.py > $OUT/${TAG}_learner_probe.json 2> $OUT/${TAG}_learner_probe.err || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_trace -o l --output-format csv -- python3 $R/tools/learner_probe.py --reps 1 > $OUT/${TAG}_trace.log 2>&1 || exit 4
echo session-done
