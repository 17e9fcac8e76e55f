"""Same bytes, same rows, same process: torch fill_ of the K = 20 int32 trajectory rows (a
one-pass linear write) and the rollout launch writing them, 3 of each, alternating.  Run under
rocprofv3 --pmc with TCC write-request / DRAM-credit-stall counters to compare how the memory
side takes the two store streams (DESIGN.md "Clocks and boxes").  Prints the HIP-event times.
"""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "ac-solver-caltech_amd"))
from bench import ms_starts  # noqa: E402
from acx import ops  # noqa: E402

K, L, B, H = 20, 36, 1 << 20, 200
dev = torch.device("cuda:0")
starts = torch.as_tensor(ms_starts(L, B)).to(dev)
state = starts.clone()
cnt = torch.zeros(B, dtype=torch.int32, device=dev)
g = torch.Generator(device=dev)
g.manual_seed(0)
acts = torch.randint(0, 12, (K, B), dtype=torch.int32, device=dev, generator=g)
obs = torch.zeros((K, B, 2 * L), dtype=torch.int32, device=dev)
rew = torch.zeros((K, B), dtype=torch.int32, device=dev)
dn = torch.zeros((K, B), dtype=torch.uint8, device=dev)
tr = torch.zeros((K, B), dtype=torch.uint8, device=dev)
plan = ops.RolloutPlan(state, starts, cnt, T=K, horizon=H, obs_traj=obs, reward_traj=rew, done_traj=dn,
                       trunc_traj=tr)
plan(acts)
torch.cuda.synchronize()
res = {"fill_ms": [], "rollout_ms": []}
for _ in range(3):
    for kind in ("fill", "rollout"):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        if kind == "fill":
            obs.fill_(1)
        else:
            state.copy_(starts)
            cnt.zero_()
            e0.record()
            plan(acts)
        e1.record()
        torch.cuda.synchronize()
        res[kind + "_ms"].append(round(e0.elapsed_time(e1), 4))
res["obs_bytes"] = obs.numel() * 4
print(json.dumps(res))
