"""GPU parity of the owner-partitioned BFS (csrc/acx_sbfs.hip, acx/search/_sharded_bfs.py):
with 1, 2 and 3 ranks (the multi-rank cases are processes sharing cuda:0 over gloo) the
results equal the reference bfs (breadth_first.py:15-97) on its own outputs
(tests/golden/kat_search*.json), and the union of the ranks' node stores, ordered by global id,
equals the single-GPU device BFS's FIFO queue node for node."""
import json
import os
import socket

import numpy as np
import pytest
import torch

from conftest import GOLDEN, PKG_ROOT, REPO

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


def _ak3(L):
    from acx.envs.utils import convert_relators_to_presentation
    return convert_relators_to_presentation([1, 1, 1, -2, -2, -2, -2], [1, 2, 1, -2, -1, -2], L)


def _ms17():
    """The Miller-Schupp start of tests/golden/search_scale.json's non-AK(3) cases (L = 36)."""
    with open(os.path.join(GOLDEN, "search_scale.json")) as f:
        return next(c["presentation"] for c in json.load(f)
                    if c["L"] == 36 and c["presentation"] != _ak3(36).tolist())


def _extra_cases(n=None):
    with open(os.path.join(GOLDEN, "kat_search_extra.json")) as f:
        cases = [c for c in json.load(f) if c["search_fn"] == "bfs"]
    return cases if n is None else cases[:n]


def _run_cases(cases, chunk, search):
    """[(ok, path, nodes at budget cut) | 'raises'] per case."""
    from acx.search import _sharded_bfs as S
    out = []
    for c in cases:
        try:
            ok, path = search(np.array(c["presentation"]), c["budget"], c["cyclical"], chunk)
        except AssertionError:
            out.append("raises")
            continue
        out.append((ok, None if path is None else [list(x) for x in path],
                    S.LAST_STATS["nodes"] if S.LAST_STATS["status"] == 2 else None))
    return out


def _sbfs(pres, budget, cyc, chunk):
    from acx.search._sharded_bfs import sharded_bfs
    return sharded_bfs(pres, budget, cyclically_reduce_after_moves=cyc, device=DEV, chunk=chunk)


def _check_cases(cases, results):
    assert len(cases) == len(results)
    for c, r in zip(cases, results):
        if c["raises"]:
            assert r == "raises", c
            continue
        ok, path, nodes = r
        assert ok == c["ok"] and path == c["path"], c
        if c["budget_nodes"] is not None:
            assert nodes == c["budget_nodes"], c


@pytest.mark.parametrize("chunk", [0, 3])
def test_sharded_bfs_one_rank_reference_searches(chunk):
    cases = _extra_cases()
    _check_cases(cases, _run_cases(cases, chunk, _sbfs))


def test_sharded_bfs_one_rank_node_order():
    from acx.search import _device_bfs as D
    from acx.search import _sharded_bfs as S
    start = _ak3(36)
    r_d = D.device_bfs(start, 200_000, device=DEV, chunk=5000, keep_node_keys=True)
    nd = D.LAST_STATS["nodes"]
    dk = D.LAST_STATS["node_keys"][:nd]
    r_s = S.sharded_bfs(start, 200_000, device=DEV, chunk=5000, keep_node_keys=True)
    assert r_s == r_d and S.LAST_STATS["nodes"] == nd
    ids, keys = S.LAST_STATS["node_ids"], S.LAST_STATS["node_keys"]
    assert np.array_equal(ids[:nd], np.arange(nd)) and np.array_equal(keys[:nd], dk)
    assert S.LAST_STATS["chunks"] == D.LAST_STATS["chunks"] and S.LAST_STATS["parents"] == D.LAST_STATS["parents"]
    assert S.LAST_STATS["min_length"] == D.LAST_STATS["min_length"]
    # AK(2) known answer (tests/search/test_bfs.py:12-17)
    with open(os.path.join(GOLDEN, "kat_search.json")) as f:
        kat = json.load(f)
    ak2 = np.array([1, 1, -2, -2, -2, 0, 0, 1, 2, 1, -2, -1, -2, 0])
    ok, path = S.sharded_bfs(ak2, int(1e6), device=DEV)
    assert [ok, [list(x) for x in path]] == kat["bfs_ak2"]


def test_sharded_bfs_arena_regrowth():
    """the key arena starting at 64 records (test hook) regrows by doubling between chunks --
    entries name arena positions, so a reallocation must leave every probe, key compare, parent
    expansion and lookup intact: same nodes in the same order as the device BFS, and the
    reference's AK(2) path"""
    import ctypes
    from acx import _lib
    from acx.search import _device_bfs as D
    from acx.search import _sharded_bfs as S
    hook = _lib.load().acx_internal_sbfs_arena_cap
    hook.argtypes = [ctypes.c_int32]
    hook.restype = None
    start = _ak3(36)
    r_d = D.device_bfs(start, 100_000, device=DEV, chunk=3000, keep_node_keys=True)
    nd = D.LAST_STATS["nodes"]
    dk = D.LAST_STATS["node_keys"][:nd]
    S.release_workspaces()
    hook(6)
    try:
        r_s = S.sharded_bfs(start, 100_000, device=DEV, chunk=3000, keep_node_keys=True)
        ids, keys, n_s = S.LAST_STATS["node_ids"], S.LAST_STATS["node_keys"], S.LAST_STATS["nodes"]
        with open(os.path.join(GOLDEN, "kat_search.json")) as f:
            kat = json.load(f)
        ak2 = np.array([1, 1, -2, -2, -2, 0, 0, 1, 2, 1, -2, -1, -2, 0])
        S.release_workspaces()
        ok, path = S.sharded_bfs(ak2, int(1e6), device=DEV)
    finally:
        hook(0)
        S.release_workspaces()
    assert r_s == r_d and n_s == nd
    assert np.array_equal(ids[:nd], np.arange(nd)) and np.array_equal(keys[:nd], dk)
    assert [ok, [list(x) for x in path]] == kat["bfs_ak2"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, jobs, q):
    import sys
    for p in (REPO, PKG_ROOT):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from acx.search import _sharded_bfs as S
        out = {}
        for name, (pres, budget, cyc, chunk) in jobs["orders"].items():
            r = S.sharded_bfs(np.array(pres), budget, verbose=True, cyclically_reduce_after_moves=cyc, device=DEV,
                              chunk=chunk, keep_node_keys=True)
            out[name] = (r, S.LAST_STATS["nodes"], S.LAST_STATS["node_ids"], S.LAST_STATS["node_keys"],
                         S.LAST_STATS["min_trace"])
        out["cases"] = _run_cases(jobs["cases"], jobs["case_chunk"], _sbfs)
        q.put((rank, out))
    except Exception as e:  # report instead of hanging the other ranks' queue reads
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4])
def test_sharded_bfs_multi_rank(world):
    import torch.multiprocessing as mp

    from acx.search import _device_bfs as D
    orders = {"ak3_36": (_ak3(36).tolist(), 150_000, False, 4096),
              "ak3_36_cyc": (_ak3(36).tolist(), 60_000, True, 777),
              "ak3_128": (_ak3(128).tolist(), 30_000, False, 0),
              "ak2": ([1, 1, -2, -2, -2, 0, 0, 1, 2, 1, -2, -1, -2, 0], 10 ** 6, False, 64),
              # a start whose search finds new minima (the verbose trace crosses the ranks)
              "ms17": (_ms17(), 60_000, False, 3000)}
    cases = _extra_cases(40)
    jobs = {"orders": orders, "cases": cases, "case_chunk": 3}
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, jobs, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    for r in range(world):
        assert not isinstance(res[r], str), res[r]
    for r in range(world):
        assert ps[r].exitcode == 0
        _check_cases(cases, res[r]["cases"])
    for name, (pres, budget, cyc, chunk) in orders.items():
        ref = D.device_bfs(np.array(pres), budget, cyclically_reduce_after_moves=cyc, device=DEV, chunk=chunk,
                           keep_node_keys=True)
        nd = D.LAST_STATS["nodes"]
        for r in range(world):  # the verbose new-minimum sequence, merged over the ranks
            assert res[r][name][4] == D.LAST_STATS["min_trace"], name
        dk = D.LAST_STATS["node_keys"]
        ids = np.concatenate([res[r][name][2] for r in range(world)])
        keys = np.concatenate([res[r][name][3] for r in range(world)])
        for r in range(world):
            assert res[r][name][0] == ref and res[r][name][1] == nd, name
        # every node stored exactly once, on its owner; ids in order = the device queue
        order = np.argsort(ids, kind="stable")
        ids, keys = ids[order], keys[order]
        # (the device BFS reports the queue up to the end of the search; the stores may also
        # hold the survivors of the last chunk after it)
        n = len(dk)
        assert n >= min(nd, 1) and len(ids) >= n and np.unique(ids).size == len(ids), name
        assert np.array_equal(ids[:n], np.arange(n)), name
        assert np.array_equal(keys[:n], dk), name


_RCCL_SCRIPT = r"""
import json, sys
sys.path[:0] = [%(repo)r, %(pkg)r, %(tests)r]
import numpy as np
import torch
import torch.distributed as dist
import bench
from conftest import state_digest, unpack_keys_np
dev = bench.dist_setup(0, 1, "nccl", force=True)   # bench.py's own multi-GPU setup, one rank
assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
bench.barrier()
assert bench.synced_max(1.5, dev) == 1.5
from acx.search import _sharded_bfs as SB
c = json.loads(sys.argv[1])
res = SB.sharded_bfs(np.array(c["presentation"]), c["budget"], cyclically_reduce_after_moves=c["cyclical"],
                     device=dev, keep_node_keys=True, always_exchange=True)
st = SB.LAST_STATS
order = np.argsort(st["node_ids"])
keys = st["node_keys"][order][: c["parents"]]
dig, cps = state_digest(unpack_keys_np(keys, c["L"]), c["checkpoints"].keys())
print(json.dumps({"exchange": st["exchange"], "parents": st["parents"], "digest": dig, "cps": cps,
                  "result": [bool(res[0]), None if res[1] is None else [list(x) for x in res[1]]]}))
SB.release_workspaces()
dist.destroy_process_group()
"""


def test_rccl_exchanges_one_rank_at_scale():
    """The RCCL code paths on hardware without a multi-GPU run: bench.py's
    multi-GPU setup (dist_setup: nccl process group bound to cuda:0 with device_id, barrier,
    max-over-ranks all_reduce) in a one-rank group, then the owner-partitioned BFS with every
    per-chunk exchange forced through _Comm's device-tensor branch (RCCL all_gather,
    all_to_all_single, all_reduce) on the AK(3) 10^6-node reference run (search_scale.json):
    the parent order digest, parent count and result equal the reference's."""
    import subprocess
    import sys
    with open(os.path.join(GOLDEN, "search_scale.json")) as f:
        c = next(x for x in json.load(f) if x["search_fn"] == "bfs" and x["L"] == 36 and not x["cyclical"]
                 and x["presentation"] == _ak3(36).tolist() and x["budget"] == 10 ** 6)
    code = _RCCL_SCRIPT % {"repo": REPO, "pkg": PKG_ROOT, "tests": os.path.join(REPO, "tests")}
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "-c", code, json.dumps(c)], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["exchange"] == "device"
    assert out["parents"] == c["parents"] and out["digest"] == c["digest"] and out["cps"] == c["checkpoints"]
    assert out["result"] == [c["ok"], c["path"]]
