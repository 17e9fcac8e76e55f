"""Driver for the device BFS (csrc/acx_bfs.hip, C-ABI acx_bfs_* in include/acx.h): the whole
search -- queue, visited set, 12-way expansion, dedup, budget -- runs on the GPU; the host
enqueues the chunks of parents one ahead without waiting between them.  Results equal
ac_solver/search/breadth_first.py:15-97 (same path, same budget cut)."""

from __future__ import annotations

import numpy as np
import torch

from .. import _lib
from ..envs.utils import is_array_valid_presentation

LAST_STATS = {}  # statistics of the most recent device search
_HANDLES = {}  # (device, L, cyclical, chunk) -> (handle, capacity)


def _handle(lib, dev: torch.device, L: int, cyclical: bool, chunk: int, max_nodes: int):
    key = (dev.index, L, bool(cyclical), int(chunk))
    h = _HANDLES.get(key)
    # reuse a workspace that is big enough but not wastefully big (a search never sees an earlier
    # one's visited set: table entries carry the search's epoch, csrc/acx_bfs.hip)
    if h is not None and h[1] >= max_nodes and (h[1] <= 16 * max_nodes or h[1] <= (1 << 20)):
        return h[0]
    if h is not None:
        lib.acx_bfs_destroy(h[0])
        del _HANDLES[key]
    cap = max(int(max_nodes), 1024)
    with torch.cuda.device(dev):
        ptr = lib.acx_bfs_create(L, cap, int(chunk), int(bool(cyclical)))
    if not ptr:
        raise _lib.ACXError(f"acx_bfs_create(L={L}, max_nodes={cap}) failed (device memory?)")
    _HANDLES[key] = (ptr, cap)
    return ptr


def release_workspaces() -> None:
    """Free the cached device workspaces."""
    lib = _lib.load()
    for ptr, _ in _HANDLES.values():
        lib.acx_bfs_destroy(ptr)
    _HANDLES.clear()


def device_bfs(presentation, max_nodes_to_explore=10000, verbose=False, cyclically_reduce_after_moves=False,
               device=None, chunk=0, keep_node_keys=False):
    """(True, path) | (False, None), as breadth_first.py:15-97.  chunk = parents per kernel
    round (0: up to 2^20).  keep_node_keys: LAST_STATS["node_keys"] = the packed keys of all
    discovered nodes in discovery (FIFO) order."""
    p = np.asarray(presentation)
    assert is_array_valid_presentation(p), f"{p} is not a valid presentation"
    if np.any(np.abs(p) > 2):
        raise ValueError("acx presentations use letters +-1 (x) and +-2 (y) only")
    L = len(p) // 2
    max_nodes = int(max_nodes_to_explore)
    if max_nodes < 1:  # the reference still expands the root once
        max_nodes = 1
    if max_nodes > (1 << 30):
        raise ValueError("device bfs supports at most 2^30 nodes")
    dev = torch.device(device if device is not None else "cuda")
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    lib = _lib.load()
    h = _handle(lib, dev, L, cyclically_reduce_after_moves, chunk, max_nodes)
    pres = np.ascontiguousarray(p, dtype=np.int32)
    cap = 1 << 16
    acts = np.zeros(cap, np.int32)
    tots = np.zeros(cap, np.int32)
    stats = np.zeros(5, np.int64)
    stream = torch.cuda.current_stream(dev).cuda_stream
    with torch.cuda.device(dev):
        st = lib.acx_bfs_run(h, pres.ctypes.data, max_nodes, acts.ctypes.data, tots.ctypes.data, cap,
                             stats.ctypes.data, stream)
    if st < 0:
        _lib.check(st, "acx_bfs_run")
    LAST_STATS.clear()
    LAST_STATS.update(nodes=int(stats[0]), parents=int(stats[1]), chunks=int(stats[2]), min_length=int(stats[3]),
                      status=int(st))
    if keep_node_keys:
        n = lib.acx_bfs_node_keys(h, None, 0, stream)
        nk = np.zeros((max(n, 0), _lib.key_words(L)), np.uint64)
        if n > 0:
            with torch.cuda.device(dev):
                r = lib.acx_bfs_node_keys(h, nk.ctypes.data, n, stream)
            if r < 0:
                _lib.check(r, "acx_bfs_node_keys")
        LAST_STATS["node_keys"] = nk
    ntr = lib.acx_bfs_min_trace(h, None, 0)
    trace = np.zeros(max(ntr, 1), np.int32)
    lib.acx_bfs_min_trace(h, trace.ctypes.data, ntr)
    LAST_STATS["min_trace"] = [int(v) for v in trace[:ntr]]
    if verbose:  # breadth_first.py:79-82, in the order the reference prints them
        for v in LAST_STATS["min_trace"]:
            print(f"New minimal length found: {v}")
    if st == _lib.BFS_MOVE_ERROR:
        raise AssertionError("bfs: a move produced an invalid presentation (utils.py:264-266)")
    if st == _lib.BFS_BUDGET:
        print(f"Exiting search as number of explored nodes = {int(stats[0])} has exceeded the limit "
              f"{max_nodes_to_explore}")
    if st == _lib.BFS_FOUND:
        n = int(stats[4])
        return True, [(int(acts[i]), int(tots[i])) for i in range(min(n, cap))]
    return False, None
