"""Owner-partitioned BFS (acx/search/_sharded_bfs.py, csrc/acx_sbfs.hip) on BASELINE config 4:
AK(3), L = 36, cyclical = False, to NODES distinct states, next to the single-GPU device BFS.

    python tools/bench_sbfs.py [NODES ...]                      # one process (exchanges are copies)
    torchrun --nproc-per-node G --master-addr 127.0.0.1 tools/bench_sbfs.py [NODES ...]
                                                                # G GPUs, RCCL ("nccl") exchanges
Rank 0 prints one JSON line: per budget the wall time of each search (best of 3 after a warmup),
the node count and whether the result and node count equal the device BFS's (world 1: also the
node order)."""
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ac-solver-caltech_amd"))
from acx.envs.utils import convert_relators_to_presentation  # noqa: E402
from acx.search import _device_bfs as D  # noqa: E402
from acx.search import _sharded_bfs as S  # noqa: E402

L = 36
budgets = [int(float(x)) for x in sys.argv[1:]] or [10 ** 7]
world = int(os.environ.get("WORLD_SIZE", "1"))
rank = int(os.environ.get("RANK", "0"))
local = int(os.environ.get("LOCAL_RANK", "0"))
dev = torch.device("cuda", local)
torch.cuda.set_device(dev)
if world > 1:
    dist.init_process_group("nccl", device_id=dev)
ak3 = convert_relators_to_presentation([1, 1, 1, -2, -2, -2, -2], [1, 2, 1, -2, -1, -2], L)


def timed(fn, reps=3):
    fn()
    best = 1e9
    for _ in range(reps):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best, r


out = {"world": world, "L": L, "start": "AK(3)", "cyclical": False}
for n in budgets:
    t_s, r_s = timed(lambda: S.sharded_bfs(ak3, n, device=dev))
    st = dict(S.LAST_STATS)
    row = {"sharded_s": t_s, "nodes": st["nodes"], "chunks": st["chunks"], "parents": st["parents"],
           "nodes_per_s": st["nodes"] / t_s}
    if rank == 0:
        t_d, r_d = timed(lambda: D.device_bfs(ak3, n, device=dev))
        row.update(device_bfs_s=t_d, same_result=r_d == r_s, same_nodes=D.LAST_STATS["nodes"] == st["nodes"])
        if world == 1:
            S.sharded_bfs(ak3, n, device=dev, keep_node_keys=True)
            D.device_bfs(ak3, n, device=dev, keep_node_keys=True)
            k = D.LAST_STATS["node_keys"]
            row["same_order"] = bool(np.array_equal(S.LAST_STATS["node_keys"][:len(k)], k))
        S.release_workspaces()
        D.release_workspaces()
    out[f"{n:.0e}"] = row
if rank == 0:
    print(json.dumps(out))
if world > 1:
    dist.destroy_process_group()
