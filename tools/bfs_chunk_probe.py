"""Device BFS wall time on AK(3), L = 36, at several chunk sizes (parents per round of kernels),
10^7 and 10^8 nodes, best of 3 after a warmup: what sets acx_bfs_create's default chunk.

    python tools/bfs_chunk_probe.py"""
import sys, time, json, torch, contextlib, io
sys.path.insert(0, "ac-solver-caltech_amd")
from acx.envs.utils import convert_relators_to_presentation
from acx.search import _device_bfs as D
dev = torch.device("cuda:0")
ak3 = convert_relators_to_presentation([1, 1, 1, -2, -2, -2, -2], [1, 2, 1, -2, -1, -2], 36)
out = {}
for n in (10**7, 10**8):
    for ch in (1 << 18, 1 << 19, 1 << 20, 1 << 21, 1 << 22):
        with contextlib.redirect_stdout(io.StringIO()):
            D.device_bfs(ak3, n, device=dev, chunk=ch)
            best = 1e9
            for _ in range(3):
                torch.cuda.synchronize(); t0 = time.perf_counter()
                D.device_bfs(ak3, n, device=dev, chunk=ch)
                torch.cuda.synchronize(); best = min(best, time.perf_counter() - t0)
        out[f"{n:.0e}_chunk{ch}"] = round(best * 1e3, 3)
        D.release_workspaces()
print(json.dumps(out))
