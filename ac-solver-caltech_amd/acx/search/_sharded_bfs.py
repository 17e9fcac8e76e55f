"""Breadth-first search over G GPUs, one process per GPU (csrc/acx_sbfs.hip, C-ABI acx_sbfs_* in
include/acx.h): the node store and the visited set are partitioned by key owner, the FIFO queue
is global and implicit (node g lives on the rank that owns its key, in ascending g).  Every rank
calls `sharded_bfs` with the same arguments (SPMD) and gets the same result, equal to
ac_solver/search/breadth_first.py:15-97 and to the single-GPU device BFS (same path, same
budget cut, same node order).

Per chunk of global parents [head, head + P) the ranks exchange, through torch.distributed
(RCCL over xGMI with the "nccl" backend; staged through host memory with "gloo"):
  1. all_gather of [success seq, move-error seq, min length, children per owner] per rank;
  2. all_to_all of the child records (packed key + seq) to their owners;
  3. all_reduce (sum) of the per-parent survivor masks.
Without an initialised process group (or with world size 1) the same code runs on one GPU with
the exchanges as local copies.
"""

from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from .. import _lib
from ..envs.utils import is_array_valid_presentation

LAST_STATS = {}  # statistics of the most recent sharded search on this rank
_HANDLES = {}  # (device, L, cyclical, chunk, local_cap, rank, world, exchange) -> handle
NONE = 0xFFFFFFFF


class _Comm:
    """The three exchanges of a chunk over a process group (or none)."""

    def __init__(self, group, dev, always=False):
        self.group = group
        self.dev = dev
        if dist.is_available() and dist.is_initialized():
            self.rank = dist.get_rank(group)
            self.world = dist.get_world_size(group)
            self.device_collectives = dist.get_backend(group) == "nccl"
        else:
            self.rank, self.world, self.device_collectives = 0, 1, True
        # `always`: run the collectives even in a one-rank group (which needs none), so the RCCL
        # device-tensor branch executes on a single GPU (tests/test_gpu_sbfs.py)
        self.local = self.world == 1 and not (always and dist.is_available() and dist.is_initialized())

    def all_gather_rows(self, row: np.ndarray) -> np.ndarray:
        """(world, n) int64: every rank's row."""
        if self.local:
            return row[None, :].copy()
        dev = self.dev if self.device_collectives else torch.device("cpu")
        t = torch.as_tensor(row, dtype=torch.int64, device=dev)
        out = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(out, t, group=self.group)
        return torch.stack(out).cpu().numpy()

    def all_to_all(self, recv: torch.Tensor, send: torch.Tensor, recv_splits, send_splits) -> None:
        if self.local:
            n = int(send_splits[0])
            recv[:n].copy_(send[:n])
            return
        if self.device_collectives:
            dist.all_to_all_single(recv, send, list(recv_splits), list(send_splits), group=self.group)
            return
        r = torch.empty(recv.shape, dtype=recv.dtype)
        dist.all_to_all_single(r, send.cpu(), list(recv_splits), list(send_splits), group=self.group)
        recv.copy_(r)

    def all_reduce_sum_(self, t: torch.Tensor) -> None:
        if self.local:
            return
        if self.device_collectives:
            dist.all_reduce(t, group=self.group)
            return
        c = t.cpu()
        dist.all_reduce(c, group=self.group)
        t.copy_(c)

    def sum_rows(self, row) -> np.ndarray:
        return self.all_gather_rows(np.asarray(row, dtype=np.int64)).sum(axis=0)

    def min_rows(self, row) -> np.ndarray:
        return self.all_gather_rows(np.asarray(row, dtype=np.int64)).min(axis=0)


def _handle(lib, dev, L, cyc, chunk, lcap, rank, world, exchange):
    key = (dev.index, L, bool(cyc), int(chunk), int(lcap), rank, world, bool(exchange))
    h = _HANDLES.get(key)
    if h is not None:
        return h
    release_workspaces()  # one workspace per process (they hold the largest buffers)
    with torch.cuda.device(dev):
        ptr = lib.acx_sbfs_create(L, int(lcap), int(chunk), int(bool(cyc)), rank, world)
    if not ptr:
        raise _lib.ACXError(f"acx_sbfs_create(L={L}, local_cap={lcap}, chunk={chunk}) failed (device memory?)")
    nrec = lib.acx_sbfs_max_records(ptr)
    kw = _lib.key_words(L)
    send = torch.empty(nrec * (kw + 1), dtype=torch.int64, device=dev)
    recv = torch.empty(nrec * (kw + 1) if exchange else 0, dtype=torch.int64, device=dev)
    mask = torch.empty(max(int(chunk), 1), dtype=torch.int32, device=dev)
    h = (ptr, send, recv, mask)
    _HANDLES[key] = h
    return h


def release_workspaces() -> None:
    lib = _lib.load()
    for ptr, *_ in _HANDLES.values():
        lib.acx_sbfs_destroy(ptr)
    _HANDLES.clear()


def local_capacity(max_nodes: int, world: int) -> int:
    """Node-store slots per rank: the rank's expected share of the max_nodes + 12 nodes a search
    can hold, with 25% + 4096 headroom for the hash partition's imbalance (a full store raises)."""
    n = int(max_nodes) + 12
    return min(n, (n + world - 1) // world * 5 // 4 + 4096)


TRACE_CAP = 512  # (seq, total) records per rank per chunk (acx_sbfs_trace; <= 2L + 1 in practice)


def _trace_chunk(lib, h, comm, buf, running, end_seq, stream, ok, agree, lines):
    """The verbose new-minimum lines of the last chunk (breadth_first.py:79-82): every rank reports
    its prefix minima among the chunk's children before end_seq; merged in sequence order they
    give the reference's sequence.  Returns the running minimum after the chunk."""
    n_raw = int(lib.acx_sbfs_trace(h, int(running), int(end_seq), buf.ctypes.data, TRACE_CAP, stream))
    ok(n_raw, "acx_sbfs_trace")
    n = min(max(n_raw, 0), TRACE_CAP)
    row = np.zeros(2 + 2 * TRACE_CAP, np.int64)
    row[0] = n
    row[1] = n_raw < 0 or n_raw > TRACE_CAP  # agreed on by every rank through the gathered rows
    row[2: 2 + 2 * n] = buf[: 2 * n]
    rows = comm.all_gather_rows(row)
    agree(int(rows[:, 1].sum()), "acx_sbfs_trace (or more than TRACE_CAP records)")
    recs = sorted((int(r[2 + 2 * i]), int(r[3 + 2 * i])) for r in rows for i in range(int(r[0])))
    for _, tot in recs:
        if tot < running:
            running = tot
            lines.append(tot)
    return running


def sharded_bfs(presentation, max_nodes_to_explore=10000, verbose=False, cyclically_reduce_after_moves=False,
                device=None, chunk=0, group=None, keep_node_keys=False, always_exchange=False):
    """(True, path) | (False, None), as breadth_first.py:15-97; SPMD over the ranks of `group`
    (default: the default process group, if initialised).  chunk = parents per round (0: 2^19).
    keep_node_keys: LAST_STATS["node_keys"] / ["node_ids"] = this rank's nodes (ascending id).
    always_exchange: run the exchanges through torch.distributed even in a one-rank group."""
    p = np.asarray(presentation)
    assert is_array_valid_presentation(p), f"{p} is not a valid presentation"
    if np.any(np.abs(p) > 2):
        raise ValueError("acx presentations use letters +-1 (x) and +-2 (y) only")
    L = len(p) // 2
    max_nodes = max(int(max_nodes_to_explore), 1)  # the reference still expands the root once
    if max_nodes > (1 << 30):
        raise ValueError("sharded bfs supports at most 2^30 nodes")
    dev = torch.device(device if device is not None else "cuda")
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    comm = _Comm(group, dev, always=always_exchange)
    chunk = int(chunk) if chunk else 1 << 19
    if not 1 <= chunk <= (1 << 19):
        raise ValueError("sharded bfs chunks are 1 .. 2^19 parents")
    lcap = local_capacity(max_nodes, comm.world)
    lib = _lib.load()
    # A failure on one rank must fail every rank at the same point, or its peers would block in
    # the next collective: local failures are recorded and agreed on through the exchanges the
    # search makes anyway (the gathered expand rows, the per-chunk status sum).
    local_err = None
    try:
        h, send, recv, gmask = _handle(lib, dev, L, cyclically_reduce_after_moves, chunk, lcap, comm.rank,
                                       comm.world, not comm.local)
    except _lib.ACXError as e:
        local_err = e
    if comm.sum_rows([local_err is not None])[0]:
        raise local_err or _lib.ACXError("sharded bfs: workspace creation failed on another rank")
    kw = _lib.key_words(L)
    rw = kw + 1
    pres = np.ascontiguousarray(p, dtype=np.int32)
    total0 = int(np.count_nonzero(pres))
    stream = torch.cuda.current_stream(dev).cuda_stream
    W = comm.world
    exp_out = np.zeros(6 + W, np.int64)  # acx_sbfs_expand's 5 + W values, then this rank's failure flag
    com_out = np.zeros(9, np.int64)  # acx_sbfs_commit's 5 values, then the chunk's expansion (4)
    trace_buf = np.zeros(2 * TRACE_CAP, np.int64)
    trace_min = total0  # breadth_first.py:59,79-82: the running minimum the verbose lines follow
    trace_lines = []
    failed = []  # (call, status) of failed C calls on this rank

    def ok(st, what):
        if st < 0:
            failed.append((what, int(st)))

    def agree(flag_sum, what):
        if flag_sum:
            if failed:
                _lib.check(failed[0][1], failed[0][0])
            raise _lib.ACXError(f"sharded bfs: {what} failed on another rank")

    with torch.cuda.device(dev):
        ok(lib.acx_sbfs_reset(h, pres.ctypes.data, stream), "acx_sbfs_reset")
        n_nodes, head, parents, chunks, min_len = 1, 0, 0, 0, total0
        status, succ_node, succ_act = _lib.BFS_EXHAUSTED, -1, -1
        while head < n_nodes:
            P = min(n_nodes - head, chunk)
            if comm.local:
                # one rank, nothing to exchange: the chunk runs on one read-back (the commit's); the
                # insert takes the chunk's first success / move error from the control block
                ok(lib.acx_sbfs_expand(h, head, P, exp_out.ctypes.data, 0, stream), "acx_sbfs_expand")
                ok(lib.acx_sbfs_insert(h, send.data_ptr(), 0, -1, gmask.data_ptr(), stream), "acx_sbfs_insert")
            else:
                ok(lib.acx_sbfs_expand(h, head, P, exp_out.ctypes.data, 1, stream), "acx_sbfs_expand")
                exp_out[5 + W] = len(failed)
                rows = comm.all_gather_rows(exp_out)  # (W, 6 + W)
                agree(rows[:, 5 + W].sum(), "a C call")
                succ_seq, err_seq = int(rows[:, 0].min()), int(rows[:, 1].min())
                chunk_min = int(rows[:, 2].min())
                send_counts = rows[comm.rank, 5 : 5 + W]
                recv_counts = rows[:, 5 + comm.rank]
                nsend, nrecv = int(send_counts.sum()), int(recv_counts.sum())
                if rows[:, 5: 5 + W].any():  # the same on every rank: skip an all-empty exchange together
                    ok(lib.acx_sbfs_pack(h, send.data_ptr(), stream), "acx_sbfs_pack")
                    comm.all_to_all(recv[:nrecv * rw], send[:nsend * rw], [int(c) * rw for c in recv_counts],
                                    [int(c) * rw for c in send_counts])
                end = min(succ_seq, err_seq)
                ok(lib.acx_sbfs_insert(h, recv.data_ptr(), nrecv, end, gmask.data_ptr(), stream), "acx_sbfs_insert")
                comm.all_reduce_sum_(gmask[:P])
            ok(lib.acx_sbfs_commit(h, gmask.data_ptr(), n_nodes, max_nodes - n_nodes, com_out.ctypes.data, stream),
               "acx_sbfs_commit")
            chunks += 1
            if comm.local:
                if failed:
                    _lib.check(failed[0][1], failed[0][0])
                if com_out[4] & 1:
                    raise _lib.ACXError("sharded bfs: hash table overflow")
                if com_out[4]:
                    raise _lib.ACXError("sharded bfs: a rank's node store or hash table is full")
                succ_seq, err_seq, chunk_min = int(com_out[5]), int(com_out[6]), int(com_out[7])
            else:
                # overflow bits (acx_sbfs_commit out[4]): bit 0 the insert's hash probe, bit 1 the commit's
                # node store / table rewrite -- decoded as the one-rank branch does
                st_rows = comm.sum_rows([int(com_out[4] & 1), int((com_out[4] >> 1) != 0), len(failed)])
                agree(st_rows[2], "a C call")
                if st_rows[0]:
                    raise _lib.ACXError("sharded bfs: hash table overflow")
                if st_rows[1]:
                    raise _lib.ACXError("sharded bfs: a rank's node store or hash table is full")
            total_new, cut_p, nodes_at_cut = int(com_out[0]), int(com_out[1]), int(com_out[2])
            cut = cut_p if cut_p >= 0 else None
            err_p = err_seq // 12 if err_seq != NONE else None
            suc_p = succ_seq // 12 if succ_seq != NONE else None
            err_first = err_p is not None and err_seq < succ_seq and (cut is None or err_p <= cut)
            succ_first = not err_first and suc_p is not None and (cut is None or suc_p <= cut)
            if verbose and chunk_min < trace_min:
                # the chunk's children the reference visits: up to (not incl.) the raising one, incl.
                # the successful one, through the cut parent, or all of them
                end_seq = (err_seq if err_first else succ_seq + 1 if succ_first else
                           12 * (cut + 1) if cut is not None else 12 * P)
                trace_min = _trace_chunk(lib, h, comm, trace_buf, trace_min, end_seq, stream, ok, agree,
                                         trace_lines)
            if err_first or succ_first or cut is not None:
                last = err_p if err_first else suc_p if succ_first else cut
                if succ_first:
                    min_len = 2
                else:
                    m = comm.min_rows([lib.acx_sbfs_min_len(h, last, stream)])[0]
                    min_len = min(min_len, int(m))
                parents += last + 1
                if err_first:
                    status = _lib.BFS_MOVE_ERROR
                elif succ_first:
                    status = _lib.BFS_FOUND
                    succ_node, succ_act = head + suc_p, succ_seq % 12
                else:
                    status = _lib.BFS_BUDGET
                    n_nodes = nodes_at_cut
                break
            min_len = min(min_len, chunk_min)
            parents += P
            n_nodes += total_new
            head += P

        path = None
        if status == _lib.BFS_FOUND:
            # walk up the parent ids; the rank that stores a node answers for it
            look = np.zeros(4, np.int64)
            edges = [(succ_act, 2)]
            g = succ_node
            while g > 0:
                ok(lib.acx_sbfs_lookup(h, g, look.ctypes.data, stream), "acx_sbfs_lookup")
                found = comm.sum_rows(look * (look[0] != 0))
                agree(comm.sum_rows([len(failed)])[0], "acx_sbfs_lookup")
                if found[0] != 1:
                    raise _lib.ACXError(f"sharded bfs: node {g} stored on {found[0]} ranks")
                edges.append((int(found[2]), int(found[3])))
                g = int(found[1])
            path = [(-1, total0)] + edges[::-1]

    LAST_STATS.clear()
    LAST_STATS.update(nodes=int(n_nodes), parents=int(parents), chunks=int(chunks), min_length=int(min_len),
                      status=int(status), rank=comm.rank, world=W,
                      exchange="local" if comm.local else "device" if comm.device_collectives else "host")
    if keep_node_keys:
        n = lib.acx_sbfs_node_keys(h, None, None, 0, stream)
        nk = np.zeros((max(n, 0), kw), np.uint64)
        ng = np.zeros(max(n, 0), np.int64)
        if n > 0:
            with torch.cuda.device(dev):
                r = lib.acx_sbfs_node_keys(h, nk.ctypes.data, ng.ctypes.data, n, stream)
            if r < 0:
                _lib.check(r, "acx_sbfs_node_keys")
        LAST_STATS["node_keys"], LAST_STATS["node_ids"] = nk, ng
    LAST_STATS["min_trace"] = list(trace_lines)
    if verbose and comm.rank == 0:
        for v in trace_lines:  # breadth_first.py:79-82 (printed before a raising move, as there)
            print(f"New minimal length found: {v}")
    if status == _lib.BFS_MOVE_ERROR:
        raise AssertionError("bfs: a move produced an invalid presentation (utils.py:264-266)")
    if status == _lib.BFS_BUDGET and comm.rank == 0:
        print(f"Exiting search as number of explored nodes = {n_nodes} has exceeded the limit "
              f"{max_nodes_to_explore}")
    if status == _lib.BFS_FOUND:
        return True, path
    return False, None
