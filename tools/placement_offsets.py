"""Is the headline rollout's speed a property of the allocation, or of where the obs trajectory sits
inside it (DESIGN.md "Placement")?

For each of `allocs` fresh (kept) flat int32 buffers of the trajectory's size plus `span` bytes,
the driver's workload (K = 20 acx_pack_actions + acx_rollout_packed over 2^20 envs, L = 36, the
bench.py batch) writes its (K, B, 2L) obs trajectory at a series of byte offsets into the buffer;
each (allocation, offset) is timed 3x with HIP events.  One JSON line per (allocation, offset) on
stderr, a summary on stdout.

    python tools/placement_offsets.py [allocs] [span_gb]
"""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ac-solver-caltech_amd"))
sys.path.insert(0, REPO)
from acx import ops  # noqa: E402
from bench import ms_starts  # noqa: E402

allocs = int(sys.argv[1]) if len(sys.argv) > 1 else 3
span = int(float(sys.argv[2]) * 2**30) if len(sys.argv) > 2 else 4 << 30
K, L, B, H = 20, 36, 1 << 20, 200
dev = torch.device("cuda:0")
starts = torch.as_tensor(ms_starts(L, B)).to(dev)
g = torch.Generator(device=dev)
g.manual_seed(0)
acts = torch.randint(0, 12, (K, B), dtype=torch.int32, device=dev, generator=g)
rew = torch.zeros((K, B), dtype=torch.int32, device=dev)
dn = torch.zeros((K, B), dtype=torch.uint8, device=dev)
tr = torch.zeros((K, B), dtype=torch.uint8, device=dev)
n_obs = K * B * 2 * L
offsets = [0, 4 << 10, 64 << 10, 1 << 20, 2 << 20, 4 << 20, 32 << 20, 256 << 20, 1 << 30, 2 << 30, span]
offsets = sorted({o for o in offsets if o <= span})
kept = []
res = []
for al in range(allocs):
    buf = torch.zeros(n_obs + span // 4, dtype=torch.int32, device=dev)
    kept.append(buf)
    for off in offsets:
        obs = buf[off // 4: off // 4 + n_obs].view(K, B, 2 * L)
        ms = []
        for rep in range(4):
            state = starts.clone()
            cnt = torch.zeros(B, dtype=torch.int32, device=dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ops.rollout(state, acts, starts, cnt, horizon=H, cyclical=True, obs_traj=obs, reward_traj=rew, done_traj=dn,
                        trunc_traj=tr)
            e1.record()
            torch.cuda.synchronize()
            if rep:
                ms.append(round(e0.elapsed_time(e1), 4))
        row = {"alloc": al, "offset_mb": off / 2**20, "ms": ms, "us_per_step": round((min(ms) - 0.11) / K * 1e3, 2),
               "va_gb": round((buf.data_ptr() + off) / 2**30, 3)}
        res.append(row)
        print(json.dumps(row), file=sys.stderr, flush=True)
print(json.dumps({"K": K, "B": B, "L": L, "rows": res}))
