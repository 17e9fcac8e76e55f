"""Measure what a plain HBM stream achieves on this GPU (torch fill_ / copy_ of large int32
buffers), to put the acx kernels' achieved GB/s next to a practically achievable figure."""
import json
import torch

dev = torch.device("cuda:0")
n = (16 << 30) // 4  # 16 GiB of int32
a = torch.empty(n, dtype=torch.int32, device=dev)
b = torch.empty(n, dtype=torch.int32, device=dev)
res = {}
for name, fn, nbytes in (("fill_write", lambda: a.fill_(7), 4 * n), ("copy_read_write", lambda: b.copy_(a), 8 * n)):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(5):
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / 1e3)
    res[name] = {"GBps": nbytes / best / 1e9, "bytes": nbytes, "best_s": best}
print(json.dumps(res))
