"""greedy_search with the reference's signature and results (ac_solver/search/greedy.py:15-121).

Best-first on (total length, path length, state tuple); the 12 children of every expanded
node come from one batched GPU launch (acx_expand12), several frontier nodes per launch, and
the host engine (csrc/acx_search.cpp) pops/dedups in exactly the reference's order."""

from __future__ import annotations

from ._engine import GREEDY, run_search


def greedy_search(presentation, max_nodes_to_explore=10000, verbose=False, cyclically_reduce_after_moves=False,
                  device=None, batch=None):
    """Returns (is_search_successful, path) with path = [(action, total_length), ...]
    starting at (-1, initial_total_length), as greedy.py:15-121."""
    return run_search(GREEDY, presentation, max_nodes_to_explore, verbose, cyclically_reduce_after_moves,
                      device=device, batch=batch)
