#!/bin/bash
# A/B session: the rollout GPU tests on the current library, then tools/ab_rollout.py over abv/*.so
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
TAG=${1:-ab}
shift
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "rollout or obs8 or int8" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_rollout.py "$@" > gpurun_out/${TAG}.json 2> gpurun_out/${TAG}.err
