#!/bin/bash
# rocprofv3 passes over a bench workload (GPU part only; the CPU baseline is skipped):
#   ./profile_cmd.sh TAG [bench args...]      default bench args: --warmup 200 (K = 200)
# --warmup 200 with the default K: the untimed warmup rollout then has the timed launch's length,
# so the rollout_kernel / pack_actions_kernel rows of --stats average two equal dispatches and
# their AverageNs is the timed launch's duration.  The driver's own command is
# `./profile_cmd.sh r02_k20 --steps 20 --warmup 5` (tools/summarize_profile.py picks the timed
# dispatch out of the per-dispatch trace either way).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
shift
ARGS=("$@")
[ ${#ARGS[@]} -eq 0 ] && ARGS=(--warmup 200)
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o bench --output-format csv -- python3 $R/bench.py --no-cpu "${ARGS[@]}" > $OUT/trace_bench.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o bench --output-format csv -- python3 $R/bench.py --no-cpu "${ARGS[@]}" > $OUT/pmc_fetch.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o bench --output-format csv -- python3 $R/bench.py --no-cpu "${ARGS[@]}" > $OUT/pmc_write.log 2>&1 || exit 3
echo profile-done
