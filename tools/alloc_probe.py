"""Does the rollout's speed depend on the process's allocation history?  Times the bench
rollout (B = 2^20, L = 36, T = 200) on fresh buffers, again after freeing them back to the
driver (empty_cache) and re-allocating, and over several rounds; prints ms per round."""
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ac-solver-caltech_amd"))
sys.path.insert(0, REPO)
from bench import ms_starts  # noqa: E402
from acx import ops  # noqa: E402

dev = torch.device("cuda:0")
L, B, T, H = 36, 1 << 20, 200, 200
starts = torch.as_tensor(ms_starts(L, B)).to(dev)
g = torch.Generator(device=dev)
g.manual_seed(0)
acts = torch.randint(0, 12, (T, B), dtype=torch.int32, device=dev, generator=g)
out = {}
t_start = time.time()
for rnd in range(int(sys.argv[1]) if len(sys.argv) > 1 else 4):
    obs = torch.zeros((T, B, 2 * L), dtype=torch.int32, device=dev)
    rew = torch.zeros((T, B), dtype=torch.int32, device=dev)
    dn = torch.zeros((T, B), dtype=torch.uint8, device=dev)
    tr = torch.zeros((T, B), dtype=torch.uint8, device=dev)
    ms = []
    for rep in range(4):
        state = starts.clone()
        cnt = torch.zeros(B, dtype=torch.int32, device=dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        ops.rollout(state, acts, starts, cnt, horizon=H, obs_traj=obs, reward_traj=rew, done_traj=dn, trunc_traj=tr)
        e1.record()
        torch.cuda.synchronize()
        ms.append(round(e0.elapsed_time(e1), 3))
    fill0 = torch.cuda.Event(enable_timing=True)
    fill1 = torch.cuda.Event(enable_timing=True)
    fill0.record()
    obs.fill_(3)
    fill1.record()
    torch.cuda.synchronize()
    out[f"round{rnd}"] = {"rollout_ms": ms, "fill_ms": round(fill0.elapsed_time(fill1), 3),
                          "t_s": round(time.time() - t_start, 2)}
    del obs, rew, dn, tr
    torch.cuda.empty_cache()
print(json.dumps(out))
