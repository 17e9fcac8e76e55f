"""Consecutive K-step rollout launches of the headline workload (2^20 envs, L = 36, int32
trajectory) timed one by one with HIP events on one stream, with and without a host
synchronisation between them: does a launch that follows another one run faster than one after
an idle gap (clock / power ramp, a warmed memory system), and by how much.

    python tools/rollout_b2b.py [--K 20] [--n 6] [--warm 200]
"""
import argparse
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "ac-solver-caltech_amd"))
from bench import ms_starts  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=20)
    ap.add_argument("--n", type=int, default=6)
    ap.add_argument("--warm", type=int, default=200)
    a = ap.parse_args()
    from acx import ops
    dev = torch.device("cuda:0")
    L, B, H, K = 36, 1 << 20, 200, a.K
    starts = torch.as_tensor(ms_starts(L, B)).to(dev)
    state = starts.clone()
    cnt = torch.zeros(B, dtype=torch.int32, device=dev)
    obs = torch.zeros((K, B, 2 * L), dtype=torch.int32, device=dev)
    rew = torch.zeros((K, B), dtype=torch.int32, device=dev)
    dn = torch.zeros((K, B), dtype=torch.uint8, device=dev)
    tr = torch.zeros((K, B), dtype=torch.uint8, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    acts = torch.randint(0, 12, (K, B), dtype=torch.int32, device=dev, generator=g)
    plan = ops.RolloutPlan(state, starts, cnt, T=K, horizon=H, cyclical=True, obs_traj=obs, reward_traj=rew,
                           done_traj=dn, trunc_traj=tr)
    for _ in range(max(a.warm // K, 1)):
        plan(acts)
    torch.cuda.synchronize()
    res = {"K": K, "B": B}
    for mode in ("synced", "back_to_back", "synced", "back_to_back"):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.n + 1)]
        torch.cuda.synchronize()
        ev[0].record()
        for i in range(a.n):
            plan(acts)
            ev[i + 1].record()
            if mode == "synced":
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        res.setdefault(mode, []).append([round(ev[i].elapsed_time(ev[i + 1]), 4) for i in range(a.n)])
    print(json.dumps(res))


if __name__ == "__main__":
    main()
