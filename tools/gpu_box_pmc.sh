#!/bin/bash
# Fast vs slow boxes under the placement counters: classify the box with a 1-s clock probe
# (K = 20 rollout median < 1.2 ms = fast), then run tools/profile_placement.sh's passes -- all of
# them on a fast box, the TCC and UTCL1 passes on a slow one.  Each GPU step under its own limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-box}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
rocm-smi --showmemvendor --showvbios --showmemorypartition > $OUT/${TAG}_box.txt 2>&1 || true
timeout -k 10 120 python -u tools/clock_probe.py --seconds 1.0 --idle 0.3 > $OUT/${TAG}_clock.json 2> $OUT/${TAG}_clock.err || exit 1
FAST=$(python -c "import json; print(1 if json.load(open('$OUT/${TAG}_clock.json'))['median_ms'] < 1.2 else 0)")
echo "fast=$FAST"
if [ "$FAST" = "1" ]; then
  bash tools/profile_placement.sh ${TAG}_fast || exit 2
else
  ONLY="tcc utcl_a" bash tools/profile_placement.sh ${TAG}_slow || exit 3
fi
echo box-pmc-done
