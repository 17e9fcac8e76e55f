"""Fast vs slow regions of one allocation under PMC counters (DESIGN.md "Placement").

In one process: a fresh buffer of the K = 20 trajectory's size + 4 GB; the headline's rollout
launch (bench.py batch: 2^20 envs, L = 36, K = 20) is timed writing its (K, B, 2L) trajectory at
byte offsets 0, 2, 4 GB (3 launches each), the slowest and the fastest offset are picked, and two
more launches go to each: slow, slow, fast, fast -- the last four rollout_kernel dispatches of the
process.  Under rocprofv3 --pmc (one process per pass, so each pass classifies its own buffer)
the summary script pairs those dispatches' counters with this JSON line (stdout).
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
buf = torch.zeros(n_obs + (1 << 30), dtype=torch.int32, device=dev)


def launch(off):
    obs = buf[off // 4: off // 4 + n_obs].view(K, B, 2 * L)
    state = starts.clone()
    cnt = torch.zeros(B, dtype=torch.int32, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    ops.rollout(state, acts, starts, cnt, horizon=H, cyclical=True, obs_traj=obs, reward_traj=rew, done_traj=dn,
                trunc_traj=tr)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


offs = [0, 2 << 30, 4 << 30]
t = {o: min(launch(o) for _ in range(3)) for o in offs}
slow, fast = max(offs, key=t.get), min(offs, key=t.get)
final = [("slow", launch(slow)), ("slow", launch(slow)), ("fast", launch(fast)), ("fast", launch(fast))]
print(json.dumps({"classify_ms": {str(o >> 30) + "GB": round(v, 4) for o, v in t.items()}, "slow_off_gb": slow >> 30,
                  "fast_off_gb": fast >> 30, "order": [k for k, _ in final], "final_ms": [round(v, 4) for _, v in final]}),
      flush=True)
