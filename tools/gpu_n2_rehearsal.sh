#!/bin/bash
# bench.py's N = 2 flow on one GPU (gloo, both ranks on cuda:0): first with a watchdog timeout so
# short that the sharded-BFS variant cannot finish (the line must still come out, with exit
# status 3 = bench.EXIT_BFS_STALL), then with the default through bench.py's own launcher
# (--gpus 2, no torchrun); in between, a rank dies inside the variant.  Each step under its own time limit, chained.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export ACX_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu --no-learner --no-step-api --bfs-timeout 0.2 > gpurun_out/n2_watchdog.json 2> gpurun_out/n2_watchdog.err
rc=$?
[ $rc -eq 1 ] || [ $rc -eq 3 ] || exit 1  # torchrun reports a failed rank as 1
echo watchdog-run-done rc=$rc; tail -c 400 gpurun_out/n2_watchdog.json
# rank 1 dies inside the sharded-BFS variant (ACX_BENCH_KILL_RANK): rank 0, blocked in the
# variant's collectives, still prints the line (its exchange fails, or torchrun's SIGTERM reaches
# LineGuard); torchrun's status is the dead rank's failure
ACX_BENCH_KILL_RANK=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 \
  bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu --no-learner --no-step-api > gpurun_out/n2_rankdeath.json 2> gpurun_out/n2_rankdeath.err
rc=$?
[ $rc -ne 0 ] && [ $rc -ne 124 ] && [ $rc -ne 137 ] || exit 3
grep -q '"value"' gpurun_out/n2_rankdeath.json || exit 4
echo rankdeath-run-done rc=$rc; tail -c 300 gpurun_out/n2_rankdeath.json
timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu --no-learner --no-step-api > gpurun_out/n2_default.json 2> gpurun_out/n2_default.err || exit 2
echo default-run-done
