"""expand12 at the config-4 scale for profiling: 10^7 parents -> packed child keys, and 10^6
parents -> int32 children (the two acx_expand12 output modes), parents = random walks from the
Miller-Schupp starts at L = 36 (cyclical=False, the search setting).  Prints kernel ms and GB/s;
run under rocprofv3 --pmc for VALU / wait-state counters."""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ac-solver-caltech_amd"))
sys.path.insert(0, REPO)
from bench import ms_starts  # noqa: E402
from acx import ops  # noqa: E402

dev = torch.device("cuda:0")
L = 36
res = {}
for name, N, mode in (("keys", 10_000_000, "keys"), ("children", 1_000_000, "children")):
    st = torch.as_tensor(ms_starts(L, N)).to(dev)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    for _ in range(20):  # move the parents off the starting set
        ops.step(st, torch.randint(0, 12, (N,), dtype=torch.int32, device=dev, generator=g), state_out=st,
                 cyclical=False)
    kw = 3
    keys = torch.empty((N, 12, kw), dtype=torch.int64, device=dev) if mode == "keys" else None
    ch = torch.empty((N, 12, 2 * L), dtype=torch.int32, device=dev) if mode == "children" else None

    lens = torch.empty((N, 12, 2), dtype=torch.int32, device=dev) if mode == "children" else None

    def run():
        if mode == "keys":
            ops.expand12(st, cyclical=False, children=False, lengths=False, keys=True, err=False, out={"keys": keys})
        else:
            ops.expand12(st, cyclical=False, children=True, lengths=True, keys=False, err=False,
                         out={"children": ch, "lengths": lens})

    run()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    bpp = 8 * L + (12 * 8 * kw if mode == "keys" else 12 * (8 * L + 8))
    res[name] = {"parents": N, "ms": best, "GBps": N * bpp / best / 1e6, "bytes_per_parent": bpp}
    del st, keys, ch, lens
print(json.dumps(res))
