"""bfs with the reference's signature and results (ac_solver/search/breadth_first.py:15-97).

engine="device" (default): the whole search runs on the GPU (csrc/acx_bfs.hip) -- queue,
  visited hash set in HBM, expansion, dedup, budget -- in chunks of parents.
engine="host": GPU expansion (acx_expand12) with the host engine (csrc/acx_search.cpp)
  replaying the FIFO/dedup/budget logic on packed keys (BASELINE config 4's "dedup on host");
  `device` may be a list of GPUs, over which each parent batch is sharded by index
  (every GPU expands a slice, the keys come back in order for the host dedup).
engine="sharded": one process per GPU (csrc/acx_sbfs.hip): node store and visited set
  partitioned by key owner over the ranks of `group` (default process group), exchanges through
  torch.distributed (RCCL all_to_all / all_reduce); every rank calls bfs with the same arguments.
Both scan children in (parent FIFO order, action 0..11) order with the reference's success
test, dedup and per-parent budget check, so paths are identical."""

from __future__ import annotations

from ._device_bfs import device_bfs
from ._engine import BFS, run_search
from ._sharded_bfs import sharded_bfs


def bfs(presentation, max_nodes_to_explore=10000, verbose=False, cyclically_reduce_after_moves=False, device=None,
        batch=None, engine="device", group=None):
    """Returns (True, path) or (False, None), as breadth_first.py:15-97."""
    if engine == "device":
        if isinstance(device, (list, tuple)):
            raise ValueError("the device BFS runs on one GPU; engine='host' shards the expansion over several")
        return device_bfs(presentation, max_nodes_to_explore, verbose, cyclically_reduce_after_moves, device=device,
                          chunk=batch or 0)
    if engine == "sharded":
        return sharded_bfs(presentation, max_nodes_to_explore, verbose, cyclically_reduce_after_moves, device=device,
                           chunk=batch or 0, group=group)
    if engine != "host":
        raise ValueError(f"engine must be 'device', 'sharded' or 'host', not {engine!r}")
    ok, path = run_search(BFS, presentation, max_nodes_to_explore, verbose, cyclically_reduce_after_moves,
                          device=device, batch=batch)
    return (True, path) if ok else (False, None)
