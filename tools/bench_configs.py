"""All five BASELINE.json configs on one GPU (configs[4] is the 8-GPU scaling config; its
per-GPU shard -- 1,048,576 envs at L = 128 -- is what is measured here).

1. [1,0,2,0], single ACEnv.step: latency of acx.ACEnv.step (launch + device->host copy)
   and parity with the reference output (tests/golden/config1.json).
2. 65,536 envs, Miller-Schupp starts, L = 36, random actions: per-call step API and
   rollout, env-steps/s.
3. 2^20 envs, L = 36, horizon 200, rollout with obs trajectory (= bench.py default).
4. AK(3) BFS to 10^7 states (tools/bench_search.py numbers are separate).
5. 2^20 envs/GPU, L = 128: step API and rollout.
"""
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ac-solver-caltech_amd"))
sys.path.insert(0, REPO)
import acx  # noqa: E402
from acx import ops  # noqa: E402
from bench import ms_starts  # noqa: E402

dev = torch.device("cuda:0")
res = {}

# config 1
env = acx.ACEnv(acx.ACEnvConfig(initial_state=[1, 0, 2, 0]))
golden = json.load(open(os.path.join(REPO, "tests", "golden", "config1.json")))
ok = True
for row in golden:
    env.reset()
    s, r, d, tr, info = env.step(row["action"])
    ok &= s.tolist() == row["state"] and r == row["reward"] and d == row["done"]
t0 = time.perf_counter()
n = 2000
for i in range(n):
    env.reset()
    env.step(i % 12)
res["config1_acenv_step"] = {"matches_reference": bool(ok), "us_per_reset_plus_step": (time.perf_counter() - t0) / n * 1e6}


def time_fn(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / 1e3)
    return best


def stepping(L, B, T, tag):
    starts = torch.as_tensor(ms_starts(L, B)).to(dev)
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    acts = torch.randint(0, 12, (T, B), dtype=torch.int32, device=dev, generator=g)
    H = 200
    venv = acx.VecACEnv(starts, horizon_length=H, device=dev)

    def steps():
        for t in range(T):
            venv.step(acts[t])

    s_api = time_fn(steps)
    obs = torch.zeros((T, B, 2 * L), dtype=torch.int32, device=dev)
    rew = torch.zeros((T, B), dtype=torch.int32, device=dev)
    dn = torch.zeros((T, B), dtype=torch.uint8, device=dev)
    tr = torch.zeros((T, B), dtype=torch.uint8, device=dev)
    s_roll = time_fn(lambda: venv.rollout(acts, obs, rew, dn, tr))
    s_noobs = time_fn(lambda: venv.rollout(acts, None, rew, dn, tr))
    res[tag] = {
        "envs": B, "L": L, "T": T,
        "step_api_env_steps_per_s": B * T / s_api, "step_api_us_per_step": s_api / T * 1e6,
        "rollout_obs_env_steps_per_s": B * T / s_roll,
        "rollout_no_obs_env_steps_per_s": B * T / s_noobs,
    }
    del obs


stepping(36, 65536, 200, "config2_65536_L36")
stepping(36, 1 << 20, 200, "config3_2p20_L36")
stepping(128, 1 << 20, 50, "config5_shard_2p20_L128")
print(json.dumps(res, indent=1))
