#!/bin/bash
# Round-5 session r: counters of the learner step kernel, fresh vs steady state (learner_probe.py --reps 1)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05r}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/${TAG}_pmc_fetch -o l --output-format csv -- python3 $R/tools/learner_probe.py --reps 1 > $OUT/${TAG}_pmc_fetch.log 2>&1 || exit 3
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/${TAG}_pmc_write -o l --output-format csv -- python3 $R/tools/learner_probe.py --reps 1 > $OUT/${TAG}_pmc_write.log 2>&1 || exit 3
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU -d $OUT/${TAG}_pmc_sq -o l --output-format csv -- python3 $R/tools/learner_probe.py --reps 1 > $OUT/${TAG}_pmc_sq.log 2>&1 || exit 4
echo session-done
