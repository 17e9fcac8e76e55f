"""bfs with the reference's signature and results (ac_solver/search/breadth_first.py:15-97).

FIFO frontier expanded in chunks of parents per GPU launch (acx_expand12); the host engine
(csrc/acx_search.cpp) scans children in (parent FIFO order, action 0..11) order with the
reference's success test, dedup and per-parent budget check, so paths are identical."""

from __future__ import annotations

from ._engine import BFS, run_search


def bfs(presentation, max_nodes_to_explore=10000, verbose=False, cyclically_reduce_after_moves=False, device=None,
        batch=None):
    """Returns (True, path) or (False, None), as breadth_first.py:15-97."""
    ok, path = run_search(BFS, presentation, max_nodes_to_explore, verbose, cyclically_reduce_after_moves,
                          device=device, batch=batch)
    return (True, path) if ok else (False, None)
