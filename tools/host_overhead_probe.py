"""Host-side cost of one per-call step (config 2: 65,536 envs, where the kernel is ~5 us): time
of torch.cuda.current_stream(), of the bare ctypes acx_step call with cached pointers, and of
VecACEnv.step, each over N calls (perf_counter, GPU work queued asynchronously)."""
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ac-solver-caltech_amd"))
sys.path.insert(0, REPO)
import acx  # noqa: E402
from bench import ms_starts  # noqa: E402

dev = torch.device("cuda:0")
B, L, N = 65536, 36, 4000
env = acx.VecACEnv(torch.as_tensor(ms_starts(L, B)).to(dev), horizon_length=200, device=dev)
a = torch.randint(0, 12, (B,), dtype=torch.int32, device=dev)
env.step(a)
torch.cuda.synchronize()
res = {}
t0 = time.perf_counter()
for _ in range(N):
    torch.cuda.current_stream(dev).cuda_stream
res["current_stream_us"] = (time.perf_counter() - t0) / N * 1e6
args = env._step_args()
lib = env._lib
s = torch.cuda.current_stream(dev).cuda_stream
t0 = time.perf_counter()
for _ in range(N):
    lib.acx_step(args[0], args[1], a.data_ptr(), args[2], args[3], args[4], args[5], args[6], args[7], args[8],
                 args[9], args[10], B, L, 200, 1, s)
torch.cuda.synchronize()
res["bare_ctypes_step_us"] = (time.perf_counter() - t0) / N * 1e6
t0 = time.perf_counter()
for _ in range(N):
    env.step(a)
torch.cuda.synchronize()
res["vecenv_step_us"] = (time.perf_counter() - t0) / N * 1e6
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
g = torch.cuda.CUDAGraph()
st = torch.cuda.Stream()
st.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(st):
    with torch.cuda.graph(g, stream=st):
        for _ in range(100):
            env.step(a)
torch.cuda.synchronize()
g.replay()
torch.cuda.synchronize()
e0.record()
g.replay()
e1.record()
torch.cuda.synchronize()
res["graph_replay_us_per_step"] = e0.elapsed_time(e1) / 100 * 1e3
# the reference's per-call APIs at B = 1: ACMove (ac_moves.py:159) and ACEnv.step (ac_env.py:91)
import numpy as np  # noqa: E402

p = np.zeros(72, np.int64)
p[:7] = [1, 1, 1, -2, -2, -2, -2]
p[36:42] = [1, 2, 1, -2, -1, -2]
acx.ACMove(5, p, 36)
t0 = time.perf_counter()
for i in range(2000):
    acx.ACMove(4 + i % 8, p, 36)
res["acmove_us"] = (time.perf_counter() - t0) / 2000 * 1e6
e = acx.ACEnv(acx.ACEnvConfig(initial_state=p))
e.step(5)
t0 = time.perf_counter()
for i in range(2000):
    e.step(4 + i % 8)
res["acenv_step_us"] = (time.perf_counter() - t0) / 2000 * 1e6
print(json.dumps(res))
