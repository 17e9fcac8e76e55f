"""Is the rollout's bimodal speed (DESIGN.md "Placement") a property of its HBM access pattern?
In each of N fresh processes: one obs buffer; the real rollout (acx pack + rollout_packed), the
same store pattern without the move compute (tools/store_pattern.hip flags NT+SCAL+LDS+PACK8) and
a linear fill, all into that buffer (best of 3 each).  One JSON line per process.

    python tools/alloc_probe5.py [N]
"""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)

CHILD = r'''
import ctypes, json, sys, torch
sys.path.insert(0, %(pkg)r); sys.path.insert(0, %(repo)r)
from bench import ms_starts
from acx import ops
sp = ctypes.CDLL(%(so)r)
sp.sp_tile.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
sp.sp_linear.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
dev = torch.device("cuda:0")
L, B, T, H = 36, 1 << 20, 200, 200
obs = torch.zeros((T, B, 2 * L), dtype=torch.int32, device=dev)
starts = torch.as_tensor(ms_starts(L, B)).to(dev)
g = torch.Generator(device=dev); g.manual_seed(0)
acts = torch.randint(0, 12, (T, B), dtype=torch.int32, device=dev, generator=g)
rew = torch.zeros((T, B), dtype=torch.int32, device=dev)
dn = torch.zeros((T, B), dtype=torch.uint8, device=dev)
tr = torch.zeros((T, B), dtype=torch.uint8, device=dev)
s = torch.cuda.current_stream(dev).cuda_stream
def timeit(fn):
    fn(); torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); e1.record(); torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    return round(best, 3)
def roll():
    state = starts.clone(); cnt = torch.zeros(B, dtype=torch.int32, device=dev)
    ops.rollout(state, acts, starts, cnt, horizon=H, obs_traj=obs, reward_traj=rew, done_traj=dn, trunc_traj=tr)
out = {"rollout": timeit(roll),
       "pattern": timeit(lambda: sp.sp_tile(obs.data_ptr(), rew.data_ptr(), dn.data_ptr(), tr.data_ptr(),
                                            acts.data_ptr(), B, T, 2 * L // 4, 83, s)),
       "fill": timeit(lambda: sp.sp_linear(obs.data_ptr(), obs.numel() * 4 // 16, 8192, s))}
out["rollout_again"] = timeit(roll)
print(json.dumps(out))
'''

if __name__ == "__main__":
    so = os.path.join(HERE, "libstore_pattern.so")
    if not os.path.exists(so):
        subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", "-o", so,
                               os.path.join(HERE, "store_pattern.hip")])
    code = CHILD % {"pkg": os.path.join(REPO, "ac-solver-caltech_amd"), "repo": REPO, "so": so}
    for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 6):
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        print(line[-1] if line else json.dumps({"error": r.stderr[-600:]}), flush=True)
