#!/bin/bash
# rocprofv3 passes over tools/bench_bfs.py (device BFS to 10^7 nodes + the expand12 keys kernel):
# kernel trace + stats, then separate PMC passes (HBM bytes, instruction / wait counters), each
# its own run as MI355X_MICROARCH.md prescribes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02}
OUT=$R/gpurun_out/prof_bfs_$TAG
mkdir -p $OUT
timeout -k 10 300 python3 $R/tools/bench_bfs.py 1e7,1e8 > $OUT/bench.json 2> $OUT/bench.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o bfs --output-format csv -- python3 $R/tools/bench_bfs.py 1e7 > $OUT/trace.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o bfs --output-format csv -- python3 $R/tools/bench_bfs.py 1e7 > $OUT/pmc_fetch.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o bfs --output-format csv -- python3 $R/tools/bench_bfs.py 1e7 > $OUT/pmc_write.log 2>&1 || exit 4
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES -d $OUT/pmc_sq -o bfs --output-format csv -- python3 $R/tools/bench_bfs.py 1e7 > $OUT/pmc_sq.log 2>&1 || exit 5
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/pmc_tcc -o bfs --output-format csv -- python3 $R/tools/bench_bfs.py 1e7 > $OUT/pmc_tcc.log 2>&1 || exit 6
echo profile-bfs-done
