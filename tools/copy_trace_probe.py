"""rocprofv3 --memory-copy-trace control case (no acx code): N device->host and M host->device
copies through torch, then exit.  Run under the profiler to see which copy directions get a
completion record on this stack (DESIGN.md "Device BFS": the BFS trace's undelivered copy
callbacks).

    rocprofv3 --kernel-trace --memory-copy-trace -d DIR -o probe --output-format csv -- python3 tools/copy_trace_probe.py 3 2
"""
import sys

import torch

n_d2h = int(sys.argv[1]) if len(sys.argv) > 1 else 3
n_h2d = int(sys.argv[2]) if len(sys.argv) > 2 else 2
x = torch.arange(1 << 20, dtype=torch.int64, device="cuda:0")
h = torch.empty(1 << 20, dtype=torch.int64).pin_memory()
for _ in range(n_h2d):
    x.copy_(h, non_blocking=False)
s = 0
for i in range(n_d2h):
    h.copy_(x, non_blocking=False)
    s += int(h[i])
torch.cuda.synchronize()
print(f"d2h {n_d2h} h2d {n_h2d} ok {s}")
