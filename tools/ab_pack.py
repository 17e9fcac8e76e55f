"""Interleaved A/B in one process: ops.rollout with the move ids read as int32 in the kernel
(pack_actions=False) vs pre-packed 8 per word (pack_actions=True, the default), at the bench
workload (B = 2^20, L = 36, T = 200, all outputs).  Times include the packing pass."""
import json
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ac-solver-caltech_amd"))
sys.path.insert(0, REPO)
from bench import ms_starts  # noqa: E402
from acx import ops  # noqa: E402

L = int(sys.argv[1]) if len(sys.argv) > 1 else 36
dev = torch.device("cuda:0")
B, T, H = 1 << 20, 200 if L == 36 else 100, 200
starts = torch.as_tensor(ms_starts(L, B)).to(dev)
g = torch.Generator(device=dev)
g.manual_seed(0)
acts = torch.randint(0, 12, (T, B), dtype=torch.int32, device=dev, generator=g)
obs = torch.zeros((T, B, 2 * L), dtype=torch.int32, device=dev)
rew = torch.zeros((T, B), dtype=torch.int32, device=dev)
dn = torch.zeros((T, B), dtype=torch.uint8, device=dev)
tr = torch.zeros((T, B), dtype=torch.uint8, device=dev)
ws = torch.empty(((T + 7) // 8, B), dtype=torch.int32, device=dev)


def run(pack):
    state = starts.clone()
    cnt = torch.zeros(B, dtype=torch.int32, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    ops.rollout(state, acts, starts, cnt, horizon=H, obs_traj=obs, reward_traj=rew, done_traj=dn, trunc_traj=tr,
                pack_actions=pack, packed_workspace=ws)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


res = {False: [], True: []}
for p in (False, True):
    run(p)
for _ in range(7):
    for p in (False, True):
        res[p].append(run(p))
print(json.dumps({("packed" if p else "int32"): {"ms_min": min(v), "ms_median": statistics.median(v)}
                  for p, v in res.items()}))
