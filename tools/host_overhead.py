import sys, time, os
sys.path.insert(0, 'ac-solver-caltech_amd'); sys.path.insert(0, '.')
import torch
from acx import ops, _lib
from bench import ms_starts
dev = torch.device('cuda:0'); B, L, T = 64, 36, 20
starts = torch.as_tensor(ms_starts(L, B)).to(dev); st = starts.clone(); cnt = torch.zeros(B, dtype=torch.int32, device=dev)
acts = torch.randint(0, 12, (T, B), dtype=torch.int32, device=dev)
obs = torch.zeros((T, B, 2 * L), dtype=torch.int32, device=dev)
rew = torch.zeros((T, B), dtype=torch.int32, device=dev); dn = torch.zeros((T, B), dtype=torch.uint8, device=dev); tr = torch.zeros_like(dn)
plan = ops.RolloutPlan(st, starts, cnt, T=T, horizon=200, obs_traj=obs, reward_traj=rew, done_traj=dn, trunc_traj=tr)
lib = _lib.load()
def t(f, n=300):
    for _ in range(20): f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n): f()
    t1 = time.perf_counter(); torch.cuda.synchronize()
    return (t1 - t0) / n * 1e6
s = torch.cuda.current_stream(dev).cuda_stream
args = plan._head + (acts.data_ptr(),) + plan._tail + (s,)
res = {
 'plan_call_us': t(lambda: plan(acts)),
 'ops_rollout_us': t(lambda: ops.rollout(st, acts, starts, cnt, horizon=200, obs_traj=obs, reward_traj=rew, done_traj=dn, trunc_traj=tr)),
 'raw_ctypes_us': t(lambda: plan._fn(*args)),
 'current_stream_us': t(lambda: torch.cuda.current_stream(dev).cuda_stream),
 'checks_us': t(lambda: (acts.shape != plan._ashape, acts.dtype != torch.int32, acts.device != dev, acts.is_contiguous())),
 'slice_us': t(lambda: acts[0:T]),
 'empty_kernel_fill_us': t(lambda: cnt.fill_(0)),
}
print(res)
