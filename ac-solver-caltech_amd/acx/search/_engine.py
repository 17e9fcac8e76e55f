"""Driver shared by greedy_search and bfs: GPU 12-way expansion (acx_expand12 -> packed
child keys) + the host search engine in libacx.so (csrc/acx_search.cpp), which replays the
reference's sequential pop / expand / dedup / budget logic on those keys."""

from __future__ import annotations

import ctypes
import time

import numpy as np
import torch

from .. import _lib, ops
from ..envs.utils import is_array_valid_presentation

BFS, GREEDY = 0, 1
LAST_STATS = {}  # engine statistics of the most recent search (rounds, expanded, pops)


def _pack_key(state: np.ndarray, L: int) -> np.ndarray:
    """Host packing of one presentation into the acx key format (acx.h: r0 codes, r1
    codes, n0, n1; codes x=0, x^-1=1, y=2, y^-1=3)."""
    kw = _lib.key_words(L)
    bits = np.zeros(kw * 64, dtype=np.uint8)
    code = {1: 0, -1: 1, 2: 2, -2: 3}
    lens = []
    for h in range(2):
        word = state[h * L : (h + 1) * L]
        n = int(np.count_nonzero(word))
        lens.append(n)
        for i in range(n):
            c = code[int(word[i])]
            bits[2 * (h * L + i)] = c & 1
            bits[2 * (h * L + i) + 1] = (c >> 1) & 1
    for j in range(8):
        bits[4 * L + j] = (lens[0] >> j) & 1
        bits[4 * L + 8 + j] = (lens[1] >> j) & 1
    words = np.packbits(bits.reshape(kw, 64)[:, ::-1], axis=1).view(">u8").reshape(kw).astype(np.uint64)
    return words


def _devices(device):
    """`device` may be one device or a list: the expansion of every parent batch is then
    sharded by parent index over those GPUs, the keys gathered in order."""
    if isinstance(device, (list, tuple)):
        devs = [torch.device(d) for d in device]
        if not devs:
            raise ValueError("empty device list")
        return devs
    return [torch.device(device if device is not None else "cuda")]


def _print_verbose_found(lib_found, h, path):
    first = np.zeros(2, np.int32)
    explored = ctypes.c_int64(0)
    lib_found(h, first.ctypes.data, ctypes.byref(explored))
    found = (np.array([first[0]], np.int8), np.array([first[1]], np.int8))
    print(f"Found {found} after exploring {explored.value} nodes")  # greedy.py:92-99
    print(f"Path to a trivial state: (tuples are of form (action, length of a state)) {path}")
    print(f"Total path length: {len(path)}")


def run_greedy_device(p, max_nodes_to_explore, verbose, cyclical, device=None, batch=None, keep_node_keys=False):
    """greedy_search on one GPU with the device visited set (csrc/acx_greedy.hip): the expansion
    rounds run in C++ (no Python per round)."""
    L = len(p) // 2
    dev = _devices(device)[0]
    lib = _lib.load()
    kw = _lib.key_words(L)
    pres = np.ascontiguousarray(p, dtype=np.int32)
    h = ctypes.c_void_p(0)
    with torch.cuda.device(dev):
        st = lib.acx_greedy_run(pres.ctypes.data, L, max(int(max_nodes_to_explore), 1), int(bool(cyclical)),
                                int(batch or 0), ctypes.byref(h))
    try:
        if st != _lib.OK:
            _lib.check(st, "acx_greedy_run")
        stats = np.zeros(13, np.int64)
        lib.acx_greedy_stats(h, stats.ctypes.data)
        budget = ctypes.c_int32(0)
        min_len = ctypes.c_int32(0)
        n_nodes = ctypes.c_int64(0)
        status = lib.acx_greedy_status(h, ctypes.byref(budget), ctypes.byref(min_len), ctypes.byref(n_nodes))
        LAST_STATS.clear()
        LAST_STATS.update(rounds=int(stats[0]), expanded=int(stats[1]), pops=int(stats[2]),
                          device_known_children=int(stats[3]), host_select_s=stats[4] / 1e9,
                          gpu_roundtrip_s=stats[5] / 1e9, host_replay_s=stats[6] / 1e9, stop_new=int(stats[7]),
                          stop_old=int(stats[8]), stop_aged=int(stats[9]), gpu_wait_s=stats[10] / 1e9,
                          host_cache_s=stats[11] / 1e9, retired_caches=int(stats[12]), nodes=int(n_nodes.value),
                          status=int(status), min_length=int(min_len.value), engine="device-visited-set")
        ntr = lib.acx_greedy_min_trace(h, None, 0)
        trace = np.zeros(max(ntr, 1), np.int32)
        lib.acx_greedy_min_trace(h, trace.ctypes.data, ntr)
        LAST_STATS["min_trace"] = [int(v) for v in trace[:ntr]]
        if keep_node_keys:
            nk = np.zeros((n_nodes.value, kw), np.uint64)
            lib.acx_greedy_node_keys(h, nk.ctypes.data, n_nodes.value)
            LAST_STATS["node_keys"] = nk
            npop = lib.acx_greedy_popped(h, None, 0)
            pops = np.zeros(max(npop, 1), np.int64)
            lib.acx_greedy_popped(h, pops.ctypes.data, npop)
            LAST_STATS["popped"] = pops[:npop]
        if verbose:  # greedy.py:86-89
            for v in LAST_STATS["min_trace"]:
                print(f"New minimal length found: {v}")
        if status == 3:
            raise AssertionError("a move produced an invalid presentation (utils.py:264-266)")
        cap = 1 << 16
        acts = np.zeros(cap, np.int32)
        tots = np.zeros(cap, np.int32)
        m = lib.acx_greedy_path(h, acts.ctypes.data, tots.ctypes.data, cap)
        path = [(int(acts[i]), int(tots[i])) for i in range(min(m, cap))]
        if verbose and status == 1:
            _print_verbose_found(lib.acx_greedy_found, h, path)
        if budget.value:
            print(f"Exiting search as number of explored nodes = {n_nodes.value} has exceeded the limit "
                  f"{max_nodes_to_explore}")
        return status == 1, path
    finally:
        if h.value:
            lib.acx_greedy_destroy(h)


def run_search(mode, presentation, max_nodes_to_explore, verbose, cyclical, device=None, batch=None,
               keep_node_keys=False, engine=None):
    p = np.asarray(presentation)
    assert is_array_valid_presentation(p), f"{p} is not a valid presentation"
    L = len(p) // 2
    if np.any(np.abs(p) > 2):
        raise ValueError("acx presentations use letters +-1 (x) and +-2 (y) only")
    if engine not in (None, "device", "host"):
        raise ValueError(f"engine must be 'device' or 'host', not {engine!r}")
    if mode == GREEDY and engine in (None, "device") and not isinstance(device, (list, tuple)):
        return run_greedy_device(p, max_nodes_to_explore, verbose, cyclical, device, batch, keep_node_keys)
    devs = _devices(device)
    lib = _lib.load()
    kw = _lib.key_words(L)
    # the start node is the (unreduced) input itself, as in the reference
    start_key = _pack_key(p.astype(np.int64), L)
    h = lib.acx_search_create(mode, L, start_key.ctypes.data, int(max_nodes_to_explore))
    if not h:
        raise _lib.ACXError("acx_search_create failed")
    if batch is None:
        batch = 65536 if mode == BFS else 512
    try:
        pinned_in = torch.empty((batch, kw), dtype=torch.int64).pin_memory()
        pinned_out = torch.empty((batch, 12, kw), dtype=torch.int64).pin_memory()
        G = len(devs)
        per = -(-batch // G)
        bufs = []
        for d in devs:
            bufs.append((torch.empty((per, kw), dtype=torch.int64, device=d),
                         torch.empty((per, 2 * L), dtype=torch.int32, device=d),
                         {"keys": torch.empty((per, 12, kw), dtype=torch.int64, device=d)}))
        status = 0
        t_gpu = 0.0
        # HIP events around each batch's kernels (unpack + expand12) on every GPU's stream: the
        # kernel-only share of gpu_roundtrip_s (which adds the H2D / D2H copies and the waits)
        kev = []
        while status == 0:
            # the engine writes the parents' keys straight into the pinned staging buffer
            n = lib.acx_search_next_batch(h, pinned_in.data_ptr(), batch)
            if n == 0:
                break
            g0 = time.perf_counter()
            # contiguous parent slices, one per GPU, launched asynchronously on each GPU's stream
            bounds = [n * g // G for g in range(G + 1)]
            for g, d in enumerate(devs):
                a, b = bounds[g], bounds[g + 1]
                if a == b:
                    continue
                dev_keys, dev_states, out = bufs[g]
                with torch.cuda.device(d):
                    dev_keys[: b - a].copy_(pinned_in[a:b], non_blocking=True)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    ops.unpack_keys(dev_keys[: b - a], L, out=dev_states[: b - a])
                    res = ops.expand12(dev_states[: b - a], cyclical=cyclical, children=False, lengths=False,
                                       keys=True, err=False, out=out)
                    e1.record()
                    kev.append((e0, e1))
                    pinned_out[a:b].copy_(res["keys"][: b - a], non_blocking=True)
            for d in devs:
                torch.cuda.synchronize(d)
            t_gpu += time.perf_counter() - g0
            status = lib.acx_search_feed(h, pinned_out.data_ptr(), n)
        st = np.zeros(6, np.int64)
        lib.acx_search_stats(h, st.ctypes.data)
        LAST_STATS.clear()
        LAST_STATS.update(rounds=int(st[0]), expanded=int(st[1]), pops=int(st[2]), host_next_s=st[3] / 1e9,
                          host_store_s=st[4] / 1e9, host_replay_s=st[5] / 1e9, gpu_roundtrip_s=t_gpu,
                          kernel_s=sum(e0.elapsed_time(e1) for e0, e1 in kev) / 1e3)
        budget = ctypes.c_int32(0)
        min_len = ctypes.c_int32(0)
        n_nodes = ctypes.c_int64(0)
        status = lib.acx_search_status(h, ctypes.byref(budget), ctypes.byref(min_len), ctypes.byref(n_nodes))
        LAST_STATS.update(nodes=int(n_nodes.value), status=int(status))
        if keep_node_keys:
            nk = np.zeros((n_nodes.value, kw), np.uint64)
            lib.acx_search_node_keys(h, nk.ctypes.data, n_nodes.value)
            LAST_STATS["node_keys"] = nk
            npop = lib.acx_search_popped(h, None, 0)
            pops = np.zeros(max(npop, 1), np.int64)
            lib.acx_search_popped(h, pops.ctypes.data, npop)
            LAST_STATS["popped"] = pops[:npop]
        ntr = lib.acx_search_min_trace(h, None, 0)
        trace = np.zeros(max(ntr, 1), np.int32)
        lib.acx_search_min_trace(h, trace.ctypes.data, ntr)
        LAST_STATS["min_trace"] = [int(v) for v in trace[:ntr]]
        LAST_STATS["min_length"] = int(min_len.value)
        if verbose:  # greedy.py:86-89 / breadth_first.py:79-82, in the reference's order
            for v in LAST_STATS["min_trace"]:
                print(f"New minimal length found: {v}")
        if status == 3:
            raise AssertionError("a move produced an invalid presentation (utils.py:264-266)")
        cap = 1 << 16
        acts = np.zeros(cap, np.int32)
        tots = np.zeros(cap, np.int32)
        m = lib.acx_search_path(h, acts.ctypes.data, tots.ctypes.data, cap)
        path = [(int(acts[i]), int(tots[i])) for i in range(min(m, cap))]
        if verbose and status == 1 and mode == GREEDY:
            _print_verbose_found(lib.acx_search_found, h, path)
        if budget.value:
            print(
                f"Exiting search as number of explored nodes = {n_nodes.value} has exceeded the limit "
                f"{max_nodes_to_explore}"
            )
        return status == 1, path
    finally:
        lib.acx_search_destroy(h)
