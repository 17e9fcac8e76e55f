"""How much of a rollout step is move compute?  B = 2^20, L = 36, K = 20 steps per launch from the
same synthetic Miller-Schupp batch as bench.py, HIP-event times (best of 4 after a warm launch):
  full      -- the headline launch (obs trajectory + reward/done/truncated)
  no_obs    -- reward/done/truncated only (the obs stores skipped: rollout_kernel<..., false>)
  bare      -- no trajectory outputs at all (state in/out and the moves)
  starts_K  -- the full launch restarted from the starting states every time (the first K steps
               of an episode, as the bench's timed launch) vs `full` continuing the episodes
Also the per-call step API in place and ping-pong (state_out != state_in) at L = 36 and 128.

    python tools/rollout_compute_probe.py"""
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
B, H, K = 1 << 20, 200, 20


def best(fn, reps=4):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return round(min(ts), 4), [round(t, 4) for t in ts]


out = {}
L = 36
starts = torch.as_tensor(ms_starts(L, B)).to(dev)
g = torch.Generator(device=dev)
g.manual_seed(0)
acts = torch.randint(0, 12, (K, B), dtype=torch.int32, device=dev, generator=g)
obs = torch.zeros((K, B, 2 * L), dtype=torch.int32, device=dev)
rew = torch.zeros((K, B), dtype=torch.int32, device=dev)
dn = torch.zeros((K, B), dtype=torch.uint8, device=dev)
tr = torch.zeros((K, B), dtype=torch.uint8, device=dev)
st = starts.clone()
cnt = torch.zeros(B, dtype=torch.int32, device=dev)


def roll(o=True, scal=True):
    ops.rollout(st, acts, starts, cnt, horizon=H, cyclical=True, obs_traj=obs if o else None,
                reward_traj=rew if scal else None, done_traj=dn if scal else None, trunc_traj=tr if scal else None)


out["full_ms"] = best(lambda: roll())
out["no_obs_ms"] = best(lambda: roll(o=False))
out["bare_ms"] = best(lambda: roll(o=False, scal=False))
out["full_again_ms"] = best(lambda: roll())


def restart():
    st.copy_(starts)
    cnt.zero_()


def roll_from_starts():
    restart()
    roll()


# the copy + zero run before the timed launch; time them alone and subtract
out["starts_K_incl_restart_ms"] = best(roll_from_starts)
out["restart_only_ms"] = best(restart)
for L2 in (36, 128):
    s2 = torch.as_tensor(ms_starts(L2, B)).to(dev)
    a = s2.clone()
    b = torch.empty_like(a)
    c2 = torch.zeros(B, dtype=torch.int32, device=dev)
    r1 = torch.empty(B, dtype=torch.int32, device=dev)
    d1 = torch.empty(B, dtype=torch.uint8, device=dev)
    t1 = torch.empty(B, dtype=torch.uint8, device=dev)
    l1 = torch.empty((B, 2), dtype=torch.int32, device=dev)
    acts2 = torch.randint(0, 12, (10, B), dtype=torch.int32, device=dev)

    def inplace():
        for t in range(10):
            ops.step(a, acts2[t], state_out=a, reset_state=s2, step_count=c2, horizon=H, cyclical=True, reward=r1,
                     done=d1, truncated=t1, lengths=l1)

    def pingpong():
        x, y = a, b
        for t in range(10):
            ops.step(x, acts2[t], state_out=y, reset_state=s2, step_count=c2, horizon=H, cyclical=True, reward=r1,
                     done=d1, truncated=t1, lengths=l1)
            x, y = y, x

    sb = 16 * L2 + 27
    for name, fn in (("inplace", inplace), ("pingpong", pingpong)):
        ms, _ = best(fn)
        out[f"step_L{L2}_{name}"] = {"ms_per_step": ms / 10, "frac": B * sb / (ms / 10 / 1e3) / 8e12}
    del s2, a, b
print(json.dumps(out))
