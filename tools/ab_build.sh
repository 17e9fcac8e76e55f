#!/bin/bash
# Build L = 36-only (or, with ONLY=L128, L = 128-only) variants of the env-step kernels (acx_kernels.hip + acx_curriculum.hip, C-ABI included)
# for in-process A/B timing (tools/ab_rollout.py), in parallel:
#   bash tools/ab_build.sh NAME "-DFLAG=.. -DFLAG2=.." [NAME2 "FLAGS2" ...]   -> abv/libacx_NAME.so (OUT=dir: another
# directory under the repo, e.g. one that travels with gpurun; abv/ does not)
# Another revision: SRC=/path/to/acx_kernels.hip bash tools/ab_build.sh NAME "" (e.g. from `git show`).
# The round-3 occupancy / tile-order / stagger hooks this was used with are in commit history
# (profiles/r03/r03l_ab*.json, DESIGN.md "Rollout: what its time is made of").
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=${OUT:-abv}
mkdir -p $R/$OUT
pids=()
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I$R/include -Wno-pass-failed \
    -DACX_ISA_${ONLY:-L36}_ONLY $flags -I$R/ac-solver-caltech_amd/csrc ${SRC:-$R/ac-solver-caltech_amd/csrc/acx_kernels.hip} $R/ac-solver-caltech_amd/csrc/acx_curriculum.hip -o $R/$OUT/libacx_$name.so &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
ls -la $R/$OUT
