"""Config 4 (BASELINE.json configs[3]) on the device BFS and the standalone expansion kernel:
AK(3), L = 36, cyclical = False.

    python tools/bench_bfs.py [NODES,...]        (default 10^7)

Per budget: the device BFS (csrc/acx_bfs.hip) to that many nodes, best of 3 wall-clock runs after
a warm-up (workspace allocated once), with its statistics; the same with the key-in-table layout
(acx_internal_bfs_layout(2)) first.  Then acx_expand12 with packed-key
output over the first 10^7 BFS nodes (the 12-way expansion kernel alone, 576 B per parent at
L = 36), best of 3 HIP-event timings.  One JSON line on stdout."""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ac-solver-caltech_amd"))
from acx import _lib, ops  # noqa: E402
from acx.envs.utils import convert_relators_to_presentation  # noqa: E402
from acx.search import _device_bfs as D  # noqa: E402

JSON_OUT, sys.stdout = sys.stdout, sys.stderr  # stdout: the JSON line only
budgets = [int(float(x)) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [10 ** 7]
L = 36
dev = torch.device("cuda:0")
ak3 = convert_relators_to_presentation([1, 1, 1, -2, -2, -2, -2], [1, 2, 1, -2, -1, -2], L)
kw = _lib.key_words(L)
res = {}
keys = None
layout_hook = _lib.load().acx_internal_bfs_layout
layout_hook.argtypes = [ctypes.c_int32]
layout_hook.restype = None
for nb in budgets:
    # the key-in-table layout (opt-in, acx_internal_bfs_layout(2)), A/B against the default below
    layout_hook(2)
    D.release_workspaces()
    D.device_bfs(ak3, nb, device=dev)
    walls8 = []
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        D.device_bfs(ak3, nb, device=dev)
        walls8.append(time.perf_counter() - t0)
    layout_hook(0)
    D.release_workspaces()
    res[f"device_bfs_keyintable_{nb:.0e}".replace("+", "")] = {"wall_ms": min(walls8) * 1e3,
                                                          "walls_ms": [w * 1e3 for w in walls8]}
    D.device_bfs(ak3, nb, device=dev, keep_node_keys=keys is None)
    if keys is None:
        keys = D.LAST_STATS["node_keys"][: min(10 ** 7, D.LAST_STATS["nodes"])]
    walls = []
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        D.device_bfs(ak3, nb, device=dev)
        walls.append(time.perf_counter() - t0)
    st = dict(D.LAST_STATS)
    best = min(walls)
    res[f"device_bfs_{nb:.0e}".replace("+", "")] = {
        "nodes": st["nodes"], "parents_expanded": st["parents"], "children": 12 * st["parents"],
        "chunks": st["chunks"], "wall_ms": best * 1e3, "walls_ms": [w * 1e3 for w in walls],
        "nodes_per_s": st["nodes"] / best, "children_per_s": 12 * st["parents"] / best, "status": st["status"]}
    D.release_workspaces()

# the 12-way expansion kernel alone: packed child keys of 10^7 parents
parents = ops.unpack_keys(torch.as_tensor(keys.view(np.int64)).to(dev), L)
N = parents.shape[0]
kout = {"keys": torch.empty((N, 12, kw), dtype=torch.int64, device=dev)}
ops.expand12(parents, cyclical=False, children=False, lengths=False, keys=True, err=False, out=kout)
torch.cuda.synchronize()
times = []
for _ in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    ops.expand12(parents, cyclical=False, children=False, lengths=False, keys=True, err=False, out=kout)
    e1.record()
    torch.cuda.synchronize()
    times.append(e0.elapsed_time(e1) / 1e3)
best = min(times)
bpp = 8 * L + 12 * kw * 8  # parent row in + 12 packed child keys out
res["expand12_keys"] = {"parents": N, "kernel_ms": best * 1e3, "children_per_s": 12 * N / best,
                        "bytes_per_parent": bpp, "GBps": N * bpp / best / 1e9, "frac": N * bpp / best / 8e12}
del kout

# children mode (full int32 children + lengths + error codes) over the first 10^6 parents:
# parent row 8L in, 12 x (8L + 8 + 1) out
M = min(N, 10 ** 6)
cout = {"children": torch.empty((M, 12, 2 * L), dtype=torch.int32, device=dev),
        "lengths": torch.empty((M, 12, 2), dtype=torch.int32, device=dev),
        "err": torch.empty((M, 12), dtype=torch.uint8, device=dev)}
ops.expand12(parents[:M], cyclical=False, children=True, lengths=True, keys=False, err=True, out=cout)
torch.cuda.synchronize()
times = []
for _ in range(5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    ops.expand12(parents[:M], cyclical=False, children=True, lengths=True, keys=False, err=True, out=cout)
    e1.record()
    torch.cuda.synchronize()
    times.append(e0.elapsed_time(e1) / 1e3)
best = min(times)
bpp = 8 * L + 12 * (8 * L + 9)
res["expand12_children"] = {"parents": M, "kernel_ms": best * 1e3, "children_per_s": 12 * M / best,
                            "bytes_per_parent": bpp, "GBps": M * bpp / best / 1e9, "frac": M * bpp / best / 8e12}
print(json.dumps(res), file=JSON_OUT)
