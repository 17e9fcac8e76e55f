"""Is the first full K-step rollout into a freshly allocated obs buffer slower than later ones?
The bench's shape: allocate + zero the (K, B, 2L) trajectory, a W-step warmup launch (writes
obs[0:W]), then timed K-step launches into the same buffer.  Per fresh buffer: HIP-event ms of
the 1st, 2nd and 3rd timed launch.

    python tools/first_launch_probe.py [trials]"""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ac-solver-caltech_amd"))
sys.path.insert(0, REPO)
from acx import ops  # noqa: E402
from bench import ms_starts  # noqa: E402

trials = int(sys.argv[1]) if len(sys.argv) > 1 else 5
L, B, H, K, W = 36, 1 << 20, 200, 20, 5
dev = torch.device("cuda:0")
starts = torch.as_tensor(ms_starts(L, B)).to(dev)
g = torch.Generator(device=dev)
g.manual_seed(0)
acts = torch.randint(0, 12, (W + 3 * K, B), dtype=torch.int32, device=dev, generator=g)
rows = []
keep = []
for trial in range(trials):
    obs = torch.empty((K, B, 2 * L), dtype=torch.int32, device=dev)
    rew = torch.empty((K, B), dtype=torch.int32, device=dev)
    dn = torch.empty((K, B), dtype=torch.uint8, device=dev)
    tr = torch.empty((K, B), dtype=torch.uint8, device=dev)
    for b in (obs, rew, dn, tr):
        b.zero_()
    st = starts.clone()
    cnt = torch.zeros(B, dtype=torch.int32, device=dev)

    def roll(a, T):
        ops.rollout(st, a, starts, cnt, horizon=H, cyclical=True, obs_traj=obs[:T], reward_traj=rew[:T],
                    done_traj=dn[:T], trunc_traj=tr[:T])

    roll(acts[:W], W)
    torch.cuda.synchronize()
    ms = []
    for r in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        roll(acts[W + r * K: W + (r + 1) * K], K)
        e1.record()
        torch.cuda.synchronize()
        ms.append(round(e0.elapsed_time(e1), 4))
    rows.append(ms)
    print(json.dumps({"trial": trial, "ms_1st_2nd_3rd": ms}), file=sys.stderr, flush=True)
    keep.append((obs, rew, dn, tr))
print(json.dumps({"K": K, "W": W, "rows": rows}))
