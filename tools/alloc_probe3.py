"""Does the first large allocation of a process run the rollout slower because of *where* it
lands?  For each ballast size X (GiB), a fresh process allocates X GiB first (kept resident),
then the (T, B, 2L) obs trajectory buffer, and times the rollout into it (best of 3).  Also
times a plain fill of the same buffer.  Prints one JSON line per ballast size.

    python tools/alloc_probe3.py 0 1 4 16 64
"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, sys, torch
sys.path.insert(0, %(pkg)r); sys.path.insert(0, %(repo)r)
from bench import ms_starts
from acx import ops
X = float(sys.argv[1])
dev = torch.device("cuda:0")
ballast = torch.empty(int(X * 2**30), dtype=torch.uint8, device=dev) if X > 0 else None
if ballast is not None:
    ballast.zero_()
L, B, T, H = 36, 1 << 20, 200, 200
obs = torch.zeros((T, B, 2 * L), dtype=torch.int32, device=dev)
starts = torch.as_tensor(ms_starts(L, B)).to(dev)
g = torch.Generator(device=dev); g.manual_seed(0)
acts = torch.randint(0, 12, (T, B), dtype=torch.int32, device=dev, generator=g)
rew = torch.zeros((T, B), dtype=torch.int32, device=dev)
dn = torch.zeros((T, B), dtype=torch.uint8, device=dev)
tr = torch.zeros((T, B), dtype=torch.uint8, device=dev)
def timeit(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); e0.record(); fn(); e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1)
def roll():
    state = starts.clone(); cnt = torch.zeros(B, dtype=torch.int32, device=dev)
    ops.rollout(state, acts, starts, cnt, horizon=H, obs_traj=obs, reward_traj=rew, done_traj=dn, trunc_traj=tr)
roll()
r = min(timeit(roll) for _ in range(3))
f = min(timeit(lambda: obs.fill_(1)) for _ in range(3))
print(json.dumps({"ballast_GiB": X, "rollout_ms": round(r, 3), "fill_ms": round(f, 3),
                  "obs_addr_GiB": round(obs.data_ptr() / 2**30, 2)}))
'''

if __name__ == "__main__":
    code = CHILD % {"pkg": os.path.join(REPO, "ac-solver-caltech_amd"), "repo": REPO}
    for x in sys.argv[1:] or ["0", "1", "4", "16", "64"]:
        r = subprocess.run([sys.executable, "-c", code, x], capture_output=True, text=True, timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        print(line[-1] if line else json.dumps({"ballast_GiB": x, "error": r.stderr[-400:]}), flush=True)
