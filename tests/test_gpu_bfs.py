"""GPU parity of the device BFS (csrc/acx_bfs.hip): results equal the reference bfs
(breadth_first.py:15-97) on the reference's own outputs (tests/golden/kat_search*.json),
and the discovered nodes equal the host engine's (pinned on CPU to the same fixtures) in
the same FIFO order, node for node, on AK(3) searches of 10^5..10^6 nodes."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


def _ak3(L):
    from acx.envs.utils import convert_relators_to_presentation
    return convert_relators_to_presentation([1, 1, 1, -2, -2, -2, -2], [1, 2, 1, -2, -1, -2], L)


@pytest.mark.parametrize("chunk", [0, 1, 3, 64, 1 << 21])
def test_device_bfs_random_reference_searches(chunk):
    from acx.search._device_bfs import LAST_STATS, device_bfs
    with open(os.path.join(GOLDEN, "kat_search_extra.json")) as f:
        cases = [c for c in json.load(f) if c["search_fn"] == "bfs"]
    assert len(cases) >= 100
    for c in cases:
        pres = np.array(c["presentation"])
        if c["raises"]:
            with pytest.raises(AssertionError):
                device_bfs(pres, c["budget"], cyclically_reduce_after_moves=c["cyclical"], device=DEV, chunk=chunk)
            continue
        ok, path = device_bfs(pres, c["budget"], cyclically_reduce_after_moves=c["cyclical"], device=DEV,
                              chunk=chunk)
        assert ok == c["ok"], c
        assert (None if path is None else [list(x) for x in path]) == c["path"], c
        if c["budget_nodes"] is not None:
            assert LAST_STATS["status"] == 2 and LAST_STATS["nodes"] == c["budget_nodes"], c


def test_device_bfs_workspace_reuse_across_epoch_wraps():
    """One workspace, 150 searches in a row (the visited set is never cleared between searches:
    entries carry a 6-bit search epoch and the table is cleared when it wraps, every 63
    searches): alternating AK(2) and AK(3) searches of several budgets keep giving the same
    results, node counts and discovered node sets as their first run, across two wraps."""
    from acx.search import _device_bfs as D
    D.release_workspaces()
    ak2 = np.array([1, 1, -2, -2, -2, 0, 0, 1, 2, 1, -2, -1, -2, 0])
    ak3 = _ak3(7)
    first = {}
    for i in range(150):
        pres, budget = [(ak2, 20_000), (ak3, 5_000), (ak2, 300), (ak3, 60_000)][i % 4]
        res = D.device_bfs(pres, budget, device=DEV, keep_node_keys=True)
        got = (res[0], None if res[1] is None else [list(x) for x in res[1]], D.LAST_STATS["nodes"],
               D.LAST_STATS["parents"], np.asarray(D.LAST_STATS["node_keys"]).tobytes())
        first.setdefault(i % 4, got)
        assert got == first[i % 4], i
    D.release_workspaces()


@pytest.mark.parametrize("chunk", [0, 5])
def test_device_bfs_kat_ak2_and_budgets(chunk):
    from acx.search._device_bfs import device_bfs
    with open(os.path.join(GOLDEN, "kat_search.json")) as f:
        kat = json.load(f)
    ak2 = np.array([1, 1, -2, -2, -2, 0, 0, 1, 2, 1, -2, -1, -2, 0])
    ok, path = device_bfs(ak2, int(1e6), device=DEV, chunk=chunk)
    assert [ok, [list(x) for x in path]] == kat["bfs_ak2"]
    assert list(device_bfs(ak2, 10, device=DEV, chunk=chunk)) == [False, None]


@pytest.mark.parametrize("L,budget,cyc,chunk", [(36, 10 ** 6, False, 0), (36, 300_000, True, 0),
                                                (36, 200_000, False, 4096), (128, 100_000, False, 0),
                                                (15, 100_000, False, 777)])
def test_device_bfs_node_order_equals_host_engine(L, budget, cyc, chunk):
    from acx.search import _device_bfs as D
    from acx.search import _engine as E
    start = _ak3(L)
    ok_h, path_h = E.run_search(E.BFS, start, budget, False, cyc, device=DEV, keep_node_keys=True)
    host = dict(E.LAST_STATS)
    ok_d, path_d = D.device_bfs(start, budget, cyclically_reduce_after_moves=cyc, device=DEV, chunk=chunk,
                                keep_node_keys=True)
    dev = dict(D.LAST_STATS)
    assert ok_d == ok_h and (path_d if ok_d else None) == (path_h if ok_h else None)
    assert dev["nodes"] == host["nodes"]
    hk, dk = host["node_keys"], dev["node_keys"][: dev["nodes"]]
    assert hk.shape == dk.shape and np.array_equal(hk, dk)


def test_device_bfs_api_edges():
    from acx import bfs
    from acx.search._device_bfs import LAST_STATS, device_bfs
    # budget 1: the root is still expanded once (breadth_first.py:91 runs after the loop)
    p = np.array([1, 1, 0, 2, 0, 0])
    assert device_bfs(p, 1, device=DEV) == (False, None)
    assert LAST_STATS["nodes"] >= 1 and LAST_STATS["parents"] == 1
    # trivial start: every child has length >= 2; [1,0,2,0]: concatenations give length 3
    ok, path = bfs(np.array([1, 0, 2, 0]), 100)
    ok_h, path_h = bfs(np.array([1, 0, 2, 0]), 100, engine="host")
    assert (ok, path) == (ok_h, path_h)
    with pytest.raises(AssertionError):
        bfs(np.array([1, 0, 0, 2]), 10)  # not a valid presentation (zero inside r0 ... r1)
    with pytest.raises(ValueError):
        bfs(np.array([3, 0, 2, 0]), 10)


@pytest.mark.parametrize("mode,budget,batch,shards", [("bfs", 200_000, 65536, 3), ("bfs", 50_000, 1000, 2),
                                                      ("greedy", 20_000, 512, 2)])
def test_host_engine_expansion_sharded_over_devices(mode, budget, batch, shards):
    """each parent batch split by index over a device list (here the one GPU listed
    several times, so the slicing/gather path runs) gives the same nodes, order and path."""
    from acx.search import _engine as E
    start = _ak3(36)
    m = E.BFS if mode == "bfs" else E.GREEDY
    ok1, path1 = E.run_search(m, start, budget, False, False, device=DEV, batch=batch, keep_node_keys=True)
    one = dict(E.LAST_STATS)
    okn, pathn = E.run_search(m, start, budget, False, False, device=[DEV] * shards, batch=batch,
                              keep_node_keys=True)
    many = dict(E.LAST_STATS)
    assert ok1 == okn and path1 == pathn
    assert one["nodes"] == many["nodes"] and np.array_equal(one["node_keys"], many["node_keys"])
    from acx import bfs
    with pytest.raises(ValueError):
        bfs(start, 10, device=[DEV, DEV])


@pytest.mark.parametrize("budget", [10 ** 6, 10 ** 7])
def test_device_bfs_leaves_the_stream_idle(budget):
    # acx_bfs_run retires every chunk it enqueued -- the speculative one after the search's end
    # included -- before it returns (breadth_first.py:91-97: the search returns with nothing
    # pending); a search that finds a path (AK(2)) as well as one cut by the budget (AK(3))
    import io
    from contextlib import redirect_stdout

    from acx.envs.utils import convert_relators_to_presentation
    from acx.search import bfs
    ak2 = convert_relators_to_presentation([1, 1, -2, -2, -2], [1, 2, 1, -2, -1, -2], 36)
    s = torch.cuda.current_stream(DEV)
    for pres in (_ak3(36), ak2):
        with redirect_stdout(io.StringIO()):
            bfs(pres, budget, device=DEV)
        assert s.query(), "work left on the caller's stream after bfs returned"
