"""Does the headline rollout's speed depend on the obs buffer's allocation (DESIGN.md "Placement")?

For each trial a fresh (T_buf, B, 2L) obs trajectory (+ reward/done/truncated) is allocated and
touched, then the driver's workload (a K-step acx_pack_actions + acx_rollout_packed launch, the
same synthetic Miller-Schupp batch as bench.py) is timed 3x with HIP events; the buffer is then
either freed (torch empty_cache: the next trial maps new memory) or kept (the next trial gets
another region).

    python tools/placement_probe.py [K] [T_buf,...] [trials] [keep|free]
One JSON line: per T_buf, per trial, ms per launch and us per env step."""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ac-solver-caltech_amd"))
sys.path.insert(0, REPO)
from acx import ops  # noqa: E402
from bench import ms_starts  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
tbufs = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [20, 200]
trials = int(sys.argv[3]) if len(sys.argv) > 3 else 4
mode = sys.argv[4] if len(sys.argv) > 4 else "free"
L, B, H = 36, 1 << 20, 200
dev = torch.device("cuda:0")
starts = torch.as_tensor(ms_starts(L, B)).to(dev)
g = torch.Generator(device=dev)
g.manual_seed(0)
acts = torch.randint(0, 12, (K, B), dtype=torch.int32, device=dev, generator=g)
out = {"K": K, "mode": mode}
kept = []
for tb in tbufs:
    rows = []
    for trial in range(trials):
        obs = torch.empty((tb, B, 2 * L), dtype=torch.int32, device=dev)
        rew = torch.empty((tb, B), dtype=torch.int32, device=dev)
        dn = torch.empty((tb, B), dtype=torch.uint8, device=dev)
        tr = torch.empty((tb, B), dtype=torch.uint8, device=dev)
        for b in (obs, rew, dn, tr):
            b.zero_()
        state = starts.clone()
        cnt = torch.zeros(B, dtype=torch.int32, device=dev)
        ms = []
        for rep in range(4):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ops.rollout(state, acts, starts, cnt, horizon=H, cyclical=True, obs_traj=obs[:K], reward_traj=rew[:K],
                        done_traj=dn[:K], trunc_traj=tr[:K])
            e1.record()
            torch.cuda.synchronize()
            if rep:
                ms.append(round(e0.elapsed_time(e1), 4))
        best = min(ms)
        rows.append({"ms": ms, "us_per_step": round((best - 0.11) / K * 1e3, 2), "addr_gb": round(obs.data_ptr() / 2**30, 1)})
        if mode == "keep":
            kept.append((obs, rew, dn, tr))
        del obs, rew, dn, tr
        if mode == "free":
            torch.cuda.empty_cache()
        print(json.dumps({"T_buf": tb, "trial": trial, **rows[-1]}), file=sys.stderr, flush=True)
    out[f"T_buf_{tb}"] = rows
print(json.dumps(out))
