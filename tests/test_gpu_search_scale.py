"""Config 4 at scale, pinned to the reference itself: tests/golden/search_scale.json holds
reference runs of bfs / greedy_search (tests/golden/make_golden.py --search-scale) -- AK(3) at
L = 36 to 10^6 nodes, cyclical variants, a Miller-Schupp start, near-full relators at L = 128 --
with the parent-expansion order as a rolling sha256 over the parent states (checkpoints at
1, 10, ..., 10^6 parents), the parent count, the verbose output and the result.

Every GPU engine is checked against them: the device BFS (csrc/acx_bfs.hip, two chunk sizes),
the host-dedup BFS and greedy over GPU expansions (csrc/acx_search.cpp + acx_expand12) and the
owner-partitioned BFS at one rank (csrc/acx_sbfs.hip); the 240 reference runs of
kat_search_extra.json go through the GPU paths too."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, state_digest, unpack_keys_np

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")

with open(os.path.join(GOLDEN, "search_scale.json")) as _f:
    SCALE = json.load(_f)
BFS_CASES = [c for c in SCALE if c["search_fn"] == "bfs"]
GREEDY_CASES = [c for c in SCALE if c["search_fn"] == "greedy_search"]


def _id(c):
    return f"L{c['L']}-n{c['budget']}-{'cyc' if c['cyclical'] else 'nocyc'}-{c['presentation'][:3]}"


def _check_order(states, c):
    assert len(states) == c["parents"], (len(states), c["parents"])
    dig, cps = state_digest(states, c["checkpoints"].keys())
    assert cps == c["checkpoints"]
    assert dig == c["digest"]


def _result(ok, path):
    return [bool(ok), None if path is None else [list(x) for x in path]]


@pytest.mark.parametrize("chunk", [0, 4099])
@pytest.mark.parametrize("c", BFS_CASES, ids=_id)
def test_device_bfs_matches_reference_at_scale(c, chunk, capsys):
    from acx.search import _device_bfs as D
    res = D.device_bfs(np.array(c["presentation"]), c["budget"], verbose=True,
                       cyclically_reduce_after_moves=c["cyclical"], device=DEV, chunk=chunk, keep_node_keys=True)
    out = capsys.readouterr().out.splitlines()
    assert out == c["stdout"]
    assert _result(*res) == [c["ok"], c["path"]]
    st = D.LAST_STATS
    assert st["parents"] == c["parents"]
    _check_order(unpack_keys_np(st["node_keys"][: c["parents"]], c["L"]), c)


@pytest.mark.parametrize("c", [c for c in BFS_CASES if c["L"] <= 43], ids=_id)
def test_device_bfs_key_in_table_layout_matches_reference(c, capsys):
    """The device BFS's second visited-set layout (opt-in through the test / A-B hook, L <= 43):
    each state's key kept in its table entry behind guard bits, so a duplicate is decided from
    the bucket line alone, against the same reference runs as the default 8-entry table
    (fingerprint + a key read from the node store)."""
    import ctypes
    from acx import _lib
    from acx.search import _device_bfs as D
    hook = _lib.load().acx_internal_bfs_layout
    hook.argtypes = [ctypes.c_int32]
    hook.restype = None
    D.release_workspaces()
    hook(2)
    try:
        res = D.device_bfs(np.array(c["presentation"]), c["budget"], verbose=True,
                           cyclically_reduce_after_moves=c["cyclical"], device=DEV, keep_node_keys=True)
    finally:
        hook(0)
        D.release_workspaces()
    out = capsys.readouterr().out.splitlines()
    assert out == c["stdout"]
    assert _result(*res) == [c["ok"], c["path"]]
    st = D.LAST_STATS
    assert st["parents"] == c["parents"]
    _check_order(unpack_keys_np(st["node_keys"][: c["parents"]], c["L"]), c)


@pytest.mark.parametrize("c", BFS_CASES, ids=_id)
def test_host_engine_bfs_matches_reference_at_scale(c, capsys):
    from acx.search import _engine as E
    ok, path = E.run_search(E.BFS, np.array(c["presentation"]), c["budget"], True, c["cyclical"], device=DEV,
                            keep_node_keys=True)
    out = capsys.readouterr().out.splitlines()
    assert out == c["stdout"]
    assert _result(ok, path if ok else None) == [c["ok"], c["path"]]
    st = E.LAST_STATS
    _check_order(unpack_keys_np(st["node_keys"][st["popped"]], c["L"]), c)


@pytest.mark.parametrize("c", BFS_CASES, ids=_id)
def test_sharded_bfs_one_rank_matches_reference_at_scale(c, capsys):
    from acx.search import _sharded_bfs as SB
    res = SB.sharded_bfs(np.array(c["presentation"]), c["budget"], verbose=True,
                         cyclically_reduce_after_moves=c["cyclical"], device=DEV, keep_node_keys=True)
    out = capsys.readouterr().out.splitlines()
    assert out == c["stdout"]
    assert _result(*res) == [c["ok"], c["path"]]
    st = SB.LAST_STATS
    assert st["parents"] == c["parents"]
    order = np.argsort(st["node_ids"])
    keys = st["node_keys"][order][: c["parents"]]
    _check_order(unpack_keys_np(keys, c["L"]), c)
    SB.release_workspaces()


@pytest.mark.parametrize("engine", ["device", "host"])
@pytest.mark.parametrize("c", GREEDY_CASES, ids=_id)
def test_greedy_matches_reference_at_scale(c, engine, capsys):
    """engine "device": csrc/acx_greedy.hip (visited set in HBM, C++-driven rounds); "host":
    csrc/acx_search.cpp over acx_expand12 launches."""
    from acx.search import _engine as E
    ok, path = E.run_search(E.GREEDY, np.array(c["presentation"]), c["budget"], True, c["cyclical"], device=DEV,
                            keep_node_keys=True, engine=engine)
    out = capsys.readouterr().out.splitlines()
    assert out == c["stdout"]
    assert [bool(ok), [list(x) for x in path]] == [c["ok"], c["path"]]
    st = E.LAST_STATS
    _check_order(unpack_keys_np(st["node_keys"][st["popped"]], c["L"]), c)


def test_reference_random_searches_through_gpu_paths():
    """kat_search_extra.json (240 reference runs, budgets 1..5000, both cyclical flags, runs that
    raise, the budget message's node count) through acx.bfs (device and host engines) and
    acx.greedy_search, i.e. with the GPU expansion."""
    import contextlib
    import io
    import re

    import acx
    with open(os.path.join(GOLDEN, "kat_search_extra.json")) as f:
        cases = json.load(f)
    for c in cases:
        pres = np.array(c["presentation"])
        fns = ([lambda **k: acx.bfs(engine="device", **k), lambda **k: acx.bfs(engine="host", **k)]
               if c["search_fn"] == "bfs" else
               [lambda **k: acx.greedy_search(engine="device", **k), lambda **k: acx.greedy_search(engine="host", **k)])
        for fn in fns:
            buf = io.StringIO()
            kw = dict(presentation=pres, max_nodes_to_explore=c["budget"], cyclically_reduce_after_moves=c["cyclical"])
            if c["raises"]:
                with pytest.raises(AssertionError), contextlib.redirect_stdout(buf):
                    fn(**kw)
                continue
            with contextlib.redirect_stdout(buf):
                ok, path = fn(**kw)
            assert _result(ok, path) == [c["ok"], c["path"]], c
            m = re.search(r"number of explored nodes = (\d+)", buf.getvalue())
            assert (int(m.group(1)) if m else None) == c["budget_nodes"], c


@pytest.mark.parametrize("batch", [1, 7, 64, 1024])
def test_greedy_device_engine_batch_sizes(batch):
    """The round size only changes how far the speculation runs ahead, never the result: AK(3)
    and a Miller-Schupp start at several batch sizes equal the reference's pop order."""
    from acx.search import _engine as E
    for c in [GREEDY_CASES[0], GREEDY_CASES[1]]:
        budget = min(c["budget"], 20000)
        ok, path = E.run_search(E.GREEDY, np.array(c["presentation"]), budget, False, c["cyclical"], device=DEV,
                                keep_node_keys=True, batch=batch)
        st = E.LAST_STATS
        states = unpack_keys_np(st["node_keys"][st["popped"]], c["L"])
        ref = next(r for r in SCALE if r["search_fn"] == "greedy_search" and r["presentation"] == c["presentation"]
                   and r["cyclical"] == c["cyclical"])
        want = {k: v for k, v in ref["checkpoints"].items() if int(k) <= len(states)}
        assert len(want) >= 3
        _, cps = state_digest(states, want.keys())
        assert cps == want, batch


def test_greedy_device_engine_aged_caches():
    """Large rounds on AK(3) to 10^6 nodes with the cache age limit lowered to 2^14 appends (test
    hook; default 2^16): many expanded nodes are popped more than 2^14 appends after their probe,
    so their cached children are retired (at a round start) or dropped (mid-replay) and
    re-expanded, and the in-flight table switches generations ~60 times; the pop order still
    equals the reference's."""
    import ctypes
    from acx import _lib
    from acx.search import _engine as E
    c = GREEDY_CASES[0]
    assert c["budget"] == 10 ** 6 and c["L"] == 36
    hook = _lib.load().acx_internal_greedy_age
    hook.argtypes = [ctypes.c_int32]
    hook.restype = None
    hook(14)
    try:
        ok, path = E.run_search(E.GREEDY, np.array(c["presentation"]), c["budget"], False, c["cyclical"], device=DEV,
                                keep_node_keys=True, batch=1024)
    finally:
        hook(0)
    st = E.LAST_STATS
    assert st["retired_caches"] > 0 and st["stop_aged"] + st["retired_caches"] > 1000
    assert [bool(ok), [list(x) for x in path]] == [c["ok"], c["path"]]
    _check_order(unpack_keys_np(st["node_keys"][st["popped"]], c["L"]), c)


@pytest.mark.parametrize("log2_age,batch", [(4, 1), (4, 64), (5, 7), (6, 1024)])
def test_greedy_device_engine_tiny_cache_age(log2_age, batch):
    """Cache age limits of 16..64 appends (test hook): nearly every replay stops at an aged cache
    and the in-flight table switches generations every few visits, so visits whose 12 appends
    cross a generation boundary happen constantly (a visit must not lose ids >= its
    probe's node count to a generation switch).  The pop order equals the reference's at every
    checkpoint the search reaches (20,000 nodes)."""
    import ctypes
    from acx import _lib
    from acx.search import _engine as E
    hook = _lib.load().acx_internal_greedy_age
    hook.argtypes = [ctypes.c_int32]
    hook.restype = None
    for c in GREEDY_CASES[:2]:
        hook(log2_age)
        try:
            ok, path = E.run_search(E.GREEDY, np.array(c["presentation"]), 20000, False, c["cyclical"], device=DEV,
                                    keep_node_keys=True, batch=batch)
        finally:
            hook(0)
        st = E.LAST_STATS
        if batch > 1:  # one parent per round is popped at once: nothing ages, only the table switches
            assert st["stop_aged"] + st["retired_caches"] > 100
        states = unpack_keys_np(st["node_keys"][st["popped"]], c["L"])
        want = {k: v for k, v in c["checkpoints"].items() if int(k) <= len(states)}
        assert len(want) >= 3
        _, cps = state_digest(states, want.keys())
        assert cps == want
        # the node set has no duplicates (a missed in-flight conflict would add one twice)
        keys = st["node_keys"]
        assert len(np.unique(keys, axis=0)) == len(keys)


def test_greedy_device_engine_grows_its_store():
    """The device store no longer allocates for the budget: a 2^36-node budget on a
    search that ends early just works (AK(2), the reference's greedy.py known answer); and a store
    forced to start at 2^10 nodes (test hook) regrows 10 times on the way to 10^6 nodes, re-entering
    the committed nodes each time, with the pop order still the reference's."""
    import ctypes
    import acx
    from acx import _lib
    from acx.search import _engine as E
    with open(os.path.join(GOLDEN, "kat_search.json")) as f:
        kat = json.load(f)
    ak2 = np.array([1, 1, -2, -2, -2, 0, 0, 1, 2, 1, -2, -1, -2, 0])
    ok, path = acx.greedy_search(ak2, max_nodes_to_explore=1 << 36, device=DEV)
    assert [ok, [list(x) for x in path]] == kat["greedy_ak2"]
    hook = _lib.load().acx_internal_greedy_init_cap
    hook.argtypes = [ctypes.c_int32]
    hook.restype = None
    c = GREEDY_CASES[0]
    hook(10)
    try:
        ok, path = E.run_search(E.GREEDY, np.array(c["presentation"]), c["budget"], False, c["cyclical"], device=DEV,
                                keep_node_keys=True)
    finally:
        hook(0)
    assert [bool(ok), [list(x) for x in path]] == [c["ok"], c["path"]]
    _check_order(unpack_keys_np(E.LAST_STATS["node_keys"][E.LAST_STATS["popped"]], c["L"]), c)


with open(os.path.join(GOLDEN, "search_scale_1e7.json")) as _f:
    CONFIG4 = json.load(_f)[0]


@pytest.mark.parametrize("engine", ["device", "sharded", "host"])
def test_config4_full_frontier_matches_reference(engine, capsys):
    """BASELINE configs[3] at its full size, pinned to the reference itself: the reference bfs
    from AK(3), L = 36, to 10^7 nodes (make_golden.py --search-scale-1e7: 1,589,594 parents
    expanded, every parent state in the rolling sha256) against the device BFS, the
    owner-partitioned BFS at one rank and the host-dedup engine (BASELINE's "dedup on host":
    GPU expansion, csrc/acx_search.cpp replaying the FIFO / dedup / budget) -- same printed
    budget message, result, parent count and parent order."""
    c = CONFIG4
    assert c["budget"] == 10 ** 7 and c["L"] == 36 and c["parents"] == 1589594
    if engine == "host":
        from acx.search import _engine as E
        res = E.run_search(E.BFS, np.array(c["presentation"]), c["budget"], True, c["cyclical"], device=DEV,
                           keep_node_keys=True)
        res = (True, res[1]) if res[0] else (False, None)
        st = dict(E.LAST_STATS, parents=len(E.LAST_STATS["popped"]))
        keys = E.LAST_STATS["node_keys"][E.LAST_STATS["popped"]][: c["parents"]]
    elif engine == "device":
        from acx.search import _device_bfs as D
        res = D.device_bfs(np.array(c["presentation"]), c["budget"], verbose=True,
                           cyclically_reduce_after_moves=c["cyclical"], device=DEV, keep_node_keys=True)
        st = D.LAST_STATS
        keys = st["node_keys"][: c["parents"]]
        D.release_workspaces()
    else:
        from acx.search import _sharded_bfs as SB
        res = SB.sharded_bfs(np.array(c["presentation"]), c["budget"], verbose=True,
                             cyclically_reduce_after_moves=c["cyclical"], device=DEV, keep_node_keys=True)
        st = SB.LAST_STATS
        order = np.argsort(st["node_ids"], kind="stable")
        keys = st["node_keys"][order][: c["parents"]]
        SB.release_workspaces()
    out = capsys.readouterr().out.splitlines()
    assert out == c["stdout"]
    assert _result(*res) == [c["ok"], c["path"]]
    assert st["parents"] == c["parents"]
    _check_order(unpack_keys_np(keys, c["L"]), c)
