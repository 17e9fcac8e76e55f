"""Where does the rollout kernel's time go?  Times acx_rollout at B = 2^20, L = 36, T = 200
with subsets of its outputs enabled (obs trajectory / reward+done+truncated / none)."""
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
L, B, T, H = 36, 1 << 20, 200, 200
starts = torch.as_tensor(ms_starts(L, B)).to(dev)
g = torch.Generator(device=dev)
g.manual_seed(0)
acts = torch.randint(0, 12, (T, B), dtype=torch.int32, device=dev, generator=g)
obs = torch.empty((T, B, 2 * L), dtype=torch.int32, device=dev)
rew = torch.empty((T, B), dtype=torch.int32, device=dev)
dn = torch.empty((T, B), dtype=torch.uint8, device=dev)
tr = torch.empty((T, B), dtype=torch.uint8, device=dev)
variants = {
    "full": dict(obs_traj=obs, reward_traj=rew, done_traj=dn, trunc_traj=tr),
    "obs_only": dict(obs_traj=obs),
    "scalars_only": dict(reward_traj=rew, done_traj=dn, trunc_traj=tr),
    "none": dict(),
}
res = {}
for rep in range(3):
    for name, kw in variants.items():
        state = starts.clone()
        cnt = torch.zeros(B, dtype=torch.int32, device=dev)
        ops.rollout(state, acts[:10], starts, cnt, horizon=H, **{k: v[:10] for k, v in kw.items()})
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.rollout(state, acts, starts, cnt, horizon=H, **kw)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        res.setdefault(name, []).append(ms)
out = {k: {"ms_min": min(v), "ms_all": v, "env_steps_per_s": B * T / (min(v) / 1e3)} for k, v in res.items()}
print(json.dumps(out, indent=1))
