#!/bin/bash
# Round-5 session o: the steady-state learner step split (tools/learner_probe.py), plain and
# under a rocprofv3 kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05o}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u tools/learner_probe.py > $OUT/${TAG}_learner_probe.json 2> $OUT/${TAG}_learner_probe.err || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_trace -o l --output-format csv -- python3 $R/tools/learner_probe.py --reps 1 > $OUT/${TAG}_trace.log 2>&1 || exit 4
echo session-done
