"""Host cost of one per-call step (ops.StepPlan) when the GPU is not the bound: B = 64 envs, so
the kernel is a few microseconds and back-to-back calls measure the host path (argument checks,
the current-stream lookup, the ctypes call, the launch).  Also the two current-stream lookups
alone.  Config 2 (65,536 envs, ~10 us kernels) is where this shows: StepPlan eager 5.0-6.2e9
against 6.5-6.9e9 from a hipGraph.

    python tools/host_overhead.py [--n 20000]
"""
import argparse
import json
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "ac-solver-caltech_amd"))
from bench import ms_starts  # noqa: E402


def per_call(fn, n):
    for _ in range(200):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return round((t1 - t0) / n * 1e6, 3), round((t2 - t0) / n * 1e6, 3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20000)
    a = ap.parse_args()
    from acx import ops

    dev = torch.device("cuda:0")
    out = {}
    out["current_stream_us"] = per_call(lambda: torch.cuda.current_stream(dev).cuda_stream, a.n)
    idx = dev.index
    out["raw_stream_us"] = per_call(lambda: torch._C._cuda_getCurrentRawStream(idx), a.n)
    for B in (64, 65536):
        L = 36
        starts = torch.as_tensor(ms_starts(L, B)).to(dev)
        st = starts.clone()
        cnt = torch.zeros(B, dtype=torch.int32, device=dev)
        rew = torch.zeros(B, dtype=torch.int32, device=dev)
        dn = torch.zeros(B, dtype=torch.uint8, device=dev)
        tr = torch.zeros(B, dtype=torch.uint8, device=dev)
        act = torch.randint(0, 12, (B,), dtype=torch.int32, device=dev)
        plan = ops.StepPlan(st, reset_state=starts, step_count=cnt, horizon=200, reward=rew, done=dn, truncated=tr)
        n = a.n if B == 64 else 2000
        out[f"stepplan_B{B}_us"] = per_call(lambda: plan(act), n)
        # the same step through the entry's own 17-argument ctypes call (what StepPlan made before
        # acx_step_plan_launch), and the plan's launch alone (no Python-side action checks)
        lib, sget = plan._lib, ops._stream
        args = (st.data_ptr(), st.data_ptr())
        tail = (starts.data_ptr(), cnt.data_ptr(), rew.data_ptr(), dn.data_ptr(), tr.data_ptr(), None, None, None,
                None, B, L, 200, 1)
        out[f"direct17_B{B}_us"] = per_call(lambda: lib.acx_step(*args, act.data_ptr(), *tail, sget(dev)), n)
        out[f"plan_launch_B{B}_us"] = per_call(lambda: lib.acx_step_plan_launch(plan._plan, act.data_ptr(), sget(dev)),
                                               n)
    out["note"] = "(host issue time per call, issue + drain per call) in microseconds"
    print(json.dumps(out))


if __name__ == "__main__":
    main()
