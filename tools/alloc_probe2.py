"""Is the rollout's speed a property of the output buffer's placement?  Allocates N obs
trajectory buffers that all stay resident, times the rollout into each, then times them all
again (interleaved) -- prints ms per buffer and the buffers' device addresses."""
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
N = int(sys.argv[1]) if len(sys.argv) > 1 else 3
starts = torch.as_tensor(ms_starts(L, B)).to(dev)
g = torch.Generator(device=dev)
g.manual_seed(0)
acts = torch.randint(0, 12, (T, B), dtype=torch.int32, device=dev, generator=g)
rew = torch.zeros((T, B), dtype=torch.int32, device=dev)
dn = torch.zeros((T, B), dtype=torch.uint8, device=dev)
tr = torch.zeros((T, B), dtype=torch.uint8, device=dev)


def roll(obs):
    state = starts.clone()
    cnt = torch.zeros(B, dtype=torch.int32, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    ops.rollout(state, acts, starts, cnt, horizon=H, obs_traj=obs, reward_traj=rew, done_traj=dn, trunc_traj=tr)
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1), 3)


bufs, first = [], []
for i in range(N):
    o = torch.zeros((T, B, 2 * L), dtype=torch.int32, device=dev)
    bufs.append(o)
    roll(o)
    first.append(min(roll(o) for _ in range(2)))
again = [[] for _ in range(N)]
for rep in range(3):
    for i, o in enumerate(bufs):
        again[i].append(roll(o))
print(json.dumps({"first": first, "again_min": [min(a) for a in again],
                  "addr_GiB": [round(o.data_ptr() / 2**30, 2) for o in bufs]}))
