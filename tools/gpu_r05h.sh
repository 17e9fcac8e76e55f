#!/bin/bash
# Round-5 session h: rocprofv3 (trace + FETCH_SIZE + WRITE_SIZE passes) of config 5's command and of
# the driver's command (profile_cmd.sh), for the per-variant byte check and the headline traffic.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash profile_cmd.sh ${1:-r05}_step128 --workload step --L 128 || exit 1
bash profile_cmd.sh ${1:-r05}_k20 --steps 20 --warmup 5 || exit 2
echo session-done
