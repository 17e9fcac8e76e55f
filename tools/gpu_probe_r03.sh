#!/bin/bash
# Short GPU call: rollout decomposition probe, then the placement PMC passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 240 python -u tools/rollout_parts.py 36 128 > $OUT/${TAG}_rollout_parts.json 2> $OUT/${TAG}_rollout_parts.err || exit 1
echo parts-done
bash tools/profile_placement.sh $TAG || exit 2
