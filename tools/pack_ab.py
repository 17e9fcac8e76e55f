"""A/B: acx_rollout with the move ids pre-packed (acx_pack_actions + acx_rollout_packed) vs read
as int32 by the rollout itself, at short launches (the driver's K = 20) and K = 200, same
buffers, alternating, B = 2^20, L = 36.  Prints one JSON line."""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ac-solver-caltech_amd"))
sys.path.insert(0, REPO)
from acx import ops  # noqa: E402
from bench import ms_starts  # noqa: E402

dev = torch.device("cuda:0")
B, L, H = 1 << 20, 36, 200
starts = torch.as_tensor(ms_starts(L, B)).to(dev)
g = torch.Generator(device=dev)
g.manual_seed(0)
res = {}
for T in (8, 20, 32, 200):
    acts = torch.randint(0, 12, (T, B), dtype=torch.int32, device=dev, generator=g)
    obs = torch.zeros((T, B, 2 * L), dtype=torch.int32, device=dev)
    rew = torch.zeros((T, B), dtype=torch.int32, device=dev)
    dn = torch.zeros((T, B), dtype=torch.uint8, device=dev)
    tr = torch.zeros((T, B), dtype=torch.uint8, device=dev)
    ws = torch.empty(((T + 7) // 8, B), dtype=torch.int32, device=dev)
    st = starts.clone()
    cnt = torch.zeros(B, dtype=torch.int32, device=dev)
    times = {True: [], False: []}
    for rep in range(6):
        for pk in (True, False):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ops.rollout(st, acts, starts, cnt, horizon=H, obs_traj=obs, reward_traj=rew, done_traj=dn,
                        trunc_traj=tr, pack_actions=pk, packed_workspace=ws)
            e1.record()
            torch.cuda.synchronize()
            times[pk].append(e0.elapsed_time(e1))
    res[f"T{T}"] = {"packed_ms": sorted(times[True])[1:4], "int32_ms": sorted(times[False])[1:4]}
    del obs, rew, dn, tr, acts
    torch.cuda.empty_cache()
print(json.dumps(res))
