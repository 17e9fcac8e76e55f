#!/bin/bash
# SQ instruction / wait counters and LDS counters for the rollout kernels (int32 and int8 obs
# trajectories) over the driver's bench command without the other variants: one rocprofv3
# --pmc pass per counter group (MI355X_MICROARCH.md), each under its own time limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02}
OUT=$R/gpurun_out/prof_rsq_$TAG
mkdir -p $OUT
ARGS=(--no-cpu --steps 20 --warmup 5 --no-step-api --no-learner --no-bfs --no-desync)
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES -d $OUT/pmc_sq -o r --output-format csv -- python3 $R/bench.py "${ARGS[@]}" > $OUT/pmc_sq.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM_WR -d $OUT/pmc_sq2 -o r --output-format csv -- python3 $R/bench.py "${ARGS[@]}" > $OUT/pmc_sq2.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o r --output-format csv -- python3 $R/bench.py "${ARGS[@]}" > $OUT/trace.log 2>&1 || exit 3
echo profile-rsq-done
