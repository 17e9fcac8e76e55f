#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_syntax
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in a b c d; do
  timeout -s KILL 60 rocprofv3 -E $R/tools/pmc_syntax/$v.yaml --pmc ACX_T TCC_EA0_WRREQ_sum -d $OUT/$v -o r --output-format csv -- python3 $R/tools/pmc_probe.py > $OUT/$v.log 2>&1
  echo "$v rc=$?"; grep -h "ACX_T\|TCC_EA0" $OUT/$v/*counter_collection.csv 2>/dev/null | cut -d, -f16,17 | head -3
done
