"""world_size-2 gloo test of bench.py's distributed plumbing (CPU): env-index shards are
disjoint and cover [0, N*B), the barrier + max-over-ranks timing reduction works."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, B, L, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, REPO)
    from bench import ms_starts
    starts = ms_starts(L, B, offset=rank * B)
    # global env ids of this shard and the presentation each starts from
    ids = torch.arange(rank * B, (rank + 1) * B)
    gathered = [torch.zeros_like(ids) for _ in range(world)]
    dist.all_gather(gathered, ids)
    dist.barrier()
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    q.put((rank, starts, torch.cat(gathered).numpy(), float(t.item())))
    dist.destroy_process_group()


def test_two_rank_sharding_gloo():
    world, B, L = 2, 2000, 36
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, B, L, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    all_ids = res[0][2]
    assert np.array_equal(np.sort(all_ids), np.arange(world * B))
    assert all(r[3] == float(world) for r in res)  # max over ranks
    import sys
    sys.path.insert(0, REPO)
    from bench import ms_starts
    full = ms_starts(L, world * B)
    assert np.array_equal(np.concatenate([r[1] for r in res]), full)


def test_data_loaders():
    import acx.data as D
    a = D.load_initial_states("all")
    s = D.load_initial_states("solved")
    assert a.shape == (1190, 36) and s.shape == (533, 36)
    b = D.load_initial_states("all", 36)
    assert b.shape == (1190, 72) and b.dtype == np.int32
    assert np.array_equal(b[:, :18], a[:, :18]) and np.array_equal(b[:, 36:54], a[:, 18:])
    from acx.envs.utils import is_array_valid_presentation
    assert all(is_array_valid_presentation(r) for r in b)


def _comm_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.join(REPO, "ac-solver-caltech_amd"))
    from acx.search._sharded_bfs import _Comm
    c = _Comm(None, torch.device("cpu"))
    rows = c.all_gather_rows(np.array([rank, 10 * rank + 1], np.int64))
    # rank r sends (r + 1) * (d + 1) records of 3 words to rank d, tagged with r and d
    send_counts = [(rank + 1) * (d + 1) for d in range(world)]
    recv_counts = [(s + 1) * (rank + 1) for s in range(world)]
    send = torch.cat([torch.full(((rank + 1) * (d + 1) * 3,), 100 * rank + d, dtype=torch.int64)
                      for d in range(world)])
    recv = torch.empty(sum(recv_counts) * 3, dtype=torch.int64)
    c.all_to_all(recv, send, [n * 3 for n in recv_counts], [n * 3 for n in send_counts])
    m = torch.tensor([1 << rank, 0, 1 << (rank + 4)], dtype=torch.int32)
    c.all_reduce_sum_(m)
    q.put((rank, rows, recv.numpy(), m.numpy(), c.min_rows([rank + 5])[0]))
    dist.destroy_process_group()


def test_sharded_bfs_exchanges_gloo():
    """The three exchanges of a sharded-BFS chunk (acx/search/_sharded_bfs.py _Comm) over a
    world_size-2 gloo group: row gather, variable-size all_to_all grouped by destination,
    mask sum (disjoint bits = OR)."""
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_comm_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, rows, recv, m, mn in res:
        assert rows.tolist() == [[0, 1], [1, 11]]
        exp = np.concatenate([np.full((s + 1) * (rank + 1) * 3, 100 * s + rank) for s in range(world)])
        assert np.array_equal(recv, exp)
        assert m.tolist() == [3, 0, 48] and mn == 5
