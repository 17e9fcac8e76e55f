"""Config 4 (BASELINE.json configs[3]): bfs 12-way neighbour expansion on AK(3), L = 36,
cyclical = False, frontier of 10^7 states.

Reports (1) end-to-end acx.bfs until 10^7 distinct states are known (GPU acx_expand12 in
batches of parents + the host engine's exact FIFO/dedup/budget replay), and (2) the
kernel alone: acx_expand12 over all 10^7 discovered states at once, packed-key output
(and full int32 children for the first 10^6 parents), and (3) the device BFS
(csrc/acx_bfs.hip: dedup on the GPU, the "next" step of SURVEY §8f) to the same 10^7 nodes,
plus optional larger budgets:  python tools/bench_search.py [NODES] [N2,N3,...]"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ac-solver-caltech_amd"))
import acx  # noqa: E402
from acx import _lib, ops  # noqa: E402
from acx.envs.utils import convert_relators_to_presentation  # noqa: E402
from acx.search import _engine  # noqa: E402

NODES = int(sys.argv[1]) if len(sys.argv) > 1 else 10 ** 7
L = 36
dev = torch.device("cuda:0")
ak3 = convert_relators_to_presentation([1, 1, 1, -2, -2, -2, -2], [1, 2, 1, -2, -1, -2], L)
lib = _lib.load()
kw = _lib.key_words(L)

# ---- (1) end-to-end BFS (same driver as acx.bfs, instrumented) ----
torch.cuda.synchronize()
t0 = time.perf_counter()
h = lib.acx_search_create(_engine.BFS, L, _engine._pack_key(ak3.astype(np.int64), L).ctypes.data, NODES)
batch = 1 << 17
parent_keys = np.zeros((batch, kw), np.uint64)
pin_in = torch.empty((batch, kw), dtype=torch.int64).pin_memory()
pin_out = torch.empty((batch, 12, kw), dtype=torch.int64).pin_memory()
dk = torch.empty((batch, kw), dtype=torch.int64, device=dev)
ds = torch.empty((batch, 2 * L), dtype=torch.int32, device=dev)
out = {"keys": torch.empty((batch, 12, kw), dtype=torch.int64, device=dev)}
expanded = 0
host_s = 0.0
gpu_s = 0.0
status = 0
while status == 0:
    n = lib.acx_search_next_batch(h, parent_keys.ctypes.data, batch)
    if n == 0:
        break
    g0 = time.perf_counter()
    pin_in[:n].numpy()[:] = parent_keys[:n].view(np.int64)
    dk[:n].copy_(pin_in[:n], non_blocking=True)
    ops.unpack_keys(dk[:n], L, out=ds[:n])
    ops.expand12(ds[:n], cyclical=False, children=False, lengths=False, keys=True, err=False, out=out)
    pin_out[:n].copy_(out["keys"][:n])
    g1 = time.perf_counter()
    status = lib.acx_search_feed(h, pin_out.data_ptr(), n)
    host_s += time.perf_counter() - g1
    gpu_s += g1 - g0
    expanded += n
wall = time.perf_counter() - t0
n_nodes = ctypes.c_int64(0)
lib.acx_search_status(h, None, None, ctypes.byref(n_nodes))
res = {"bfs_end_to_end": {"nodes": n_nodes.value, "parents_requested": expanded, "children": 12 * expanded,
                          "wall_s": wall, "gpu_side_s": gpu_s, "host_engine_s": host_s,
                          "children_per_s": 12 * expanded / wall, "status": int(status)}}

# ---- (2) kernel only: expand all discovered states at once ----
N = min(n_nodes.value, NODES)
keys = np.zeros((N, kw), np.uint64)
lib.acx_search_node_keys(h, keys.ctypes.data, N)
lib.acx_search_destroy(h)
dkeys = torch.as_tensor(keys.view(np.int64)).to(dev)
parents = ops.unpack_keys(dkeys, L)
kout = {"keys": torch.empty((N, 12, kw), dtype=torch.int64, device=dev)}
ops.expand12(parents, cyclical=False, children=False, lengths=False, keys=True, err=False, out=kout)
torch.cuda.synchronize()
best = 1e9
for _ in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    ops.expand12(parents, cyclical=False, children=False, lengths=False, keys=True, err=False, out=kout)
    e1.record()
    torch.cuda.synchronize()
    best = min(best, e0.elapsed_time(e1) / 1e3)
bytes_keys = N * (8 * L + 12 * kw * 8)  # parents in + packed child keys out
res["expand12_keys"] = {"parents": N, "children": 12 * N, "kernel_ms": best * 1e3, "children_per_s": 12 * N / best,
                        "GBps": bytes_keys / best / 1e9, "bytes_per_parent": 8 * L + 12 * kw * 8}
M = min(N, 10 ** 6)
cout = {"children": torch.empty((M, 12, 2 * L), dtype=torch.int32, device=dev),
        "lengths": torch.empty((M, 12, 2), dtype=torch.int32, device=dev)}
ops.expand12(parents[:M], cyclical=False, children=True, lengths=True, keys=False, err=False, out=cout)
torch.cuda.synchronize()
best = 1e9
for _ in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    ops.expand12(parents[:M], cyclical=False, children=True, lengths=True, keys=False, err=False, out=cout)
    e1.record()
    torch.cuda.synchronize()
    best = min(best, e0.elapsed_time(e1) / 1e3)
b = M * (8 * L + 12 * (8 * L + 8))
res["expand12_children"] = {"parents": M, "kernel_ms": best * 1e3, "children_per_s": 12 * M / best,
                            "GBps": b / best / 1e9, "bytes_per_parent": 8 * L + 12 * (8 * L + 8)}

# ---- (3) device BFS (csrc/acx_bfs.hip): queue, visited set, dedup, budget all on the GPU ----
from acx.search import _device_bfs as D  # noqa: E402

for n_nodes_dev in [NODES] + ([int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else []):
    D.device_bfs(ak3, n_nodes_dev, device=dev)  # allocate the workspace, warm up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ok, _ = D.device_bfs(ak3, n_nodes_dev, device=dev)
    wall = time.perf_counter() - t0
    st = dict(D.LAST_STATS)
    res[f"device_bfs_{n_nodes_dev:.0e}".replace("+", "")] = {
        "nodes": st["nodes"], "parents_expanded": st["parents"], "children": 12 * st["parents"],
        "chunks": st["chunks"], "wall_s": wall, "children_per_s": 12 * st["parents"] / wall,
        "nodes_per_s": st["nodes"] / wall, "status": st["status"],
        "speedup_vs_host_dedup": res["bfs_end_to_end"]["wall_s"] / wall if n_nodes_dev == NODES else None}
    D.release_workspaces()
print(json.dumps(res))
