#!/bin/bash
# PMC passes over tools/placement_pmc.py (fast vs slow region of one allocation): per-TCC-instance
# and per-XCC write requests (derived counters in tools/pmc_instances.yaml), write stalls, TCC tag
# stalls, DRAM credit stalls and the UTCL1 translation counters.  One rocprofv3 process per pass,
# each under its own time limit, chained.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03}
OUT=$R/gpurun_out/prof_place_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() {  # name counters...   (ONLY="name ...": just those passes)
  local n=$1; shift
  if [ -n "$ONLY" ] && [[ " $ONLY " != *" $n "* ]]; then return 0; fi
  timeout -s KILL 90 rocprofv3 -E $R/tools/pmc_instances.yaml --pmc "$@" -d $OUT/$n -o r --output-format csv -- python3 $R/tools/placement_pmc.py > $OUT/$n.log 2>&1
}
run inst ACX_WRREQ_I0 ACX_WRREQ_I1 ACX_WRREQ_I2 ACX_WRREQ_I3 ACX_WRREQ_I4 ACX_WRREQ_I5 ACX_WRREQ_I6 ACX_WRREQ_I7 ACX_WRREQ_I8 ACX_WRREQ_I9 ACX_WRREQ_I10 ACX_WRREQ_I11 ACX_WRREQ_I12 ACX_WRREQ_I13 ACX_WRREQ_I14 ACX_WRREQ_I15 || exit 1
run xcc ACX_WRREQ_X0 ACX_WRREQ_X1 ACX_WRREQ_X2 ACX_WRREQ_X3 ACX_WRREQ_X4 ACX_WRREQ_X5 ACX_WRREQ_X6 ACX_WRREQ_X7 || exit 2
run stall_inst ACX_WRSTALL_I0 ACX_WRSTALL_I1 ACX_WRSTALL_I2 ACX_WRSTALL_I3 ACX_WRSTALL_I4 ACX_WRSTALL_I5 ACX_WRSTALL_I6 ACX_WRSTALL_I7 ACX_WRSTALL_I8 ACX_WRSTALL_I9 ACX_WRSTALL_I10 ACX_WRSTALL_I11 ACX_WRSTALL_I12 ACX_WRSTALL_I13 ACX_WRSTALL_I14 ACX_WRSTALL_I15 || exit 3
run tcc TCC_EA0_WRREQ_sum TCC_TAG_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum || exit 4
run utcl_a TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS TCP_UTCL1_STALL_INFLIGHT_MAX TCP_UTCL1_STALL_MULTI_MISS || exit 5
run utcl_b TCP_UTCL1_THRASHING_STALL TCP_UTCL1_LFIFO_FULL TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS TCP_UTCL1_SERIALIZATION_STALL || exit 6
run grbm GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE || exit 7
echo placement-pmc-done
