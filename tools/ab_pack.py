"""In-process A/B of the rollout's two move-id paths: acx_pack_actions + acx_rollout_packed
(ops.rollout's default) against acx_rollout reading the (T, B) int32 ids itself, on the bench's
rollout (2^20 envs, L = 36, Miller-Schupp starts, horizon 200) with int32 and int8 obs
trajectories, the SAME buffers, interleaved, HIP events on the current stream; outputs compared.

    python tools/ab_pack.py [--K 20,200] [--reps 7]
"""
import argparse
import json
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "ac-solver-caltech_amd"))
from bench import ms_starts  # noqa: E402
from acx import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", default="20,200")
    ap.add_argument("--reps", type=int, default=7)
    a = ap.parse_args()
    Ks = [int(x) for x in a.K.split(",")]
    B, L, H, dev = 1 << 20, 36, 200, torch.device("cuda:0")
    starts = torch.as_tensor(ms_starts(L, B)).to(dev)
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    Kmax = max(Ks)
    acts = torch.randint(0, 12, (Kmax, B), dtype=torch.int32, device=dev, generator=g)
    rew = torch.zeros((Kmax, B), dtype=torch.int32, device=dev)
    dn = torch.zeros((Kmax, B), dtype=torch.uint8, device=dev)
    tr = torch.zeros((Kmax, B), dtype=torch.uint8, device=dev)
    err = torch.zeros(B, dtype=torch.uint8, device=dev)
    ec = torch.zeros(1, dtype=torch.int32, device=dev)
    obs = {"i32": torch.zeros((Kmax, B, 2 * L), dtype=torch.int32, device=dev),
           "i8": torch.zeros((Kmax, B, 2 * L), dtype=torch.int8, device=dev)}
    state = torch.empty_like(starts)
    cnt = torch.zeros(B, dtype=torch.int32, device=dev)
    res = {}
    sums = {}
    for rep in range(a.reps + 1):
        for K in Ks:
            for kind, o in obs.items():
                for pack in (True, False):
                    state.copy_(starts)
                    cnt.zero_()
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    ops.rollout(state, acts[:K], starts, cnt, horizon=H, cyclical=True, obs_traj=o[:K],
                                reward_traj=rew[:K], done_traj=dn[:K], trunc_traj=tr[:K], err=err, err_count=ec,
                                pack_actions=pack)
                    e1.record()
                    torch.cuda.synchronize()
                    key = f"K{K}_{kind}_{'packed' if pack else 'int32ids'}"
                    if rep:
                        res.setdefault(key, []).append(e0.elapsed_time(e1))
                    else:
                        sums[key] = [sum(int(o[t].view(torch.int32).sum(dtype=torch.int64)) for t in range(K)),
                                     int(state.sum(dtype=torch.int64)), int(rew[:K].sum(dtype=torch.int64)),
                                     int(cnt.sum(dtype=torch.int64))]
    out = {"ms_median": {k: statistics.median(v) for k, v in res.items()}, "ms_all": res, "checksums": sums}
    for K in Ks:
        for kind in obs:
            p, u = sums[f"K{K}_{kind}_packed"], sums[f"K{K}_{kind}_int32ids"]
            out[f"K{K}_{kind}_outputs_equal"] = p == u
    print(json.dumps(out))


if __name__ == "__main__":
    main()
