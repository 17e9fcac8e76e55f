"""Where does the PPO learner step's time go?  LearnerEnv.step at B = 2^20, L = 36 (the
bench's learner_step variant): GPU time per step (HIP events over K steps) and host time per
Python call (perf_counter, no sync).  Run under rocprofv3 --kernel-trace --stats for the
per-kernel split."""
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ac-solver-caltech_amd"))
sys.path.insert(0, REPO)
from bench import ms_starts  # noqa: E402
from acx.agents import LearnerEnv  # noqa: E402

dev = torch.device("cuda:0")
L, B, K, H = 36, 1 << 20, 50, 200
lenv = LearnerEnv(np.concatenate([ms_starts(L, B), ms_starts(L, 4096, offset=B)]), B, horizon_length=H, device=dev)
obs = torch.zeros((K + 1, B, 2 * L), dtype=torch.float32, device=dev)
rew = torch.zeros((K, B), dtype=torch.float32, device=dev)
dn = torch.zeros((K, B), dtype=torch.float32, device=dev)
g = torch.Generator(device=dev)
g.manual_seed(0)
acts = torch.randint(0, 12, (K, B), dtype=torch.int64, device=dev, generator=g)
for t in range(3):
    lenv.step(acts[t], obs_out=obs[t + 1], reward_out=rew[t], done_out=dn[t])
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
host = []
e0.record()
for t in range(K):
    h0 = time.perf_counter()
    lenv.step(acts[t], obs_out=obs[t + 1], reward_out=rew[t], done_out=dn[t])
    host.append(time.perf_counter() - h0)
e1.record()
torch.cuda.synchronize()
print(json.dumps({"event_ms_per_step": e0.elapsed_time(e1) / K, "host_ms_per_call_median": 1e3 * float(np.median(host))}))
