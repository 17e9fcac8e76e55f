"""greedy_search with the reference's signature and results (ac_solver/search/greedy.py:15-121).

Best-first on (total length, path length, state tuple), popped / deduplicated in exactly the
reference's order.
engine="device" (default, one GPU): csrc/acx_greedy.hip -- C++-driven rounds that expand the
  smallest unexpanded frontier nodes on the GPU and probe every child against the visited set
  kept in HBM; the host checks only the children the device did not know against the nodes
  appended since (the in-flight conflicts).
engine="host" (or `device` a list of GPUs): acx_expand12 launches from Python with the host
  engine (csrc/acx_search.cpp) holding the whole visited set; the expansion of each batch is
  sharded by parent index over the listed GPUs."""

from __future__ import annotations

from ._engine import GREEDY, run_search


def greedy_search(presentation, max_nodes_to_explore=10000, verbose=False, cyclically_reduce_after_moves=False,
                  device=None, batch=None, engine="device"):
    """Returns (is_search_successful, path) with path = [(action, total_length), ...]
    starting at (-1, initial_total_length), as greedy.py:15-121."""
    return run_search(GREEDY, presentation, max_nodes_to_explore, verbose, cyclically_reduce_after_moves,
                      device=device, batch=batch, engine=engine)
