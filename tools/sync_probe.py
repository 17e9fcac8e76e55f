"""How much of the driver's timed region is host synchronisation: the headline launch (2^20 envs,
L = 36, K = 20, int32 trajectory) bracketed exactly as bench.py's timed() does, wall vs HIP-event
time, with HIP's default device scheduling or with hipDeviceScheduleSpin (--spin: set through
hipSetDeviceFlags before torch creates the context).

    python tools/sync_probe.py [--spin] [--reps 9]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "ac-solver-caltech_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spin", action="store_true")
    ap.add_argument("--reps", type=int, default=9)
    a = ap.parse_args()
    if a.spin:
        hip = ctypes.CDLL("libamdhip64.so")
        assert hip.hipSetDeviceFlags(ctypes.c_uint(1)) == 0  # hipDeviceScheduleSpin
    import torch
    from bench import ms_starts
    from acx import ops
    L, B, K, H = 36, 1 << 20, 20, 200
    dev = torch.device("cuda:0")
    starts = torch.as_tensor(ms_starts(L, B)).to(dev)
    state, count = starts.clone(), torch.zeros(B, dtype=torch.int32, device=dev)
    obs = torch.empty((K, B, 2 * L), dtype=torch.int32, device=dev)
    rew = torch.empty((K, B), dtype=torch.int32, device=dev)
    dn = torch.empty((K, B), dtype=torch.uint8, device=dev)
    tr = torch.empty((K, B), dtype=torch.uint8, device=dev)
    acts = torch.randint(0, 12, (K, B), dtype=torch.int32, device=dev)
    plan = ops.RolloutPlan(state, starts, count, T=K, horizon=H, cyclical=True, obs_traj=obs, reward_traj=rew,
                           done_traj=dn, trunc_traj=tr)
    plan(acts)
    walls, evs = [], []
    for _ in range(a.reps):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        plan(acts)
        e1.record()
        torch.cuda.synchronize()
        walls.append((time.perf_counter() - t0) * 1e3)
        evs.append(e0.elapsed_time(e1))
    print(json.dumps({"spin": a.spin, "wall_ms": round(statistics.median(walls), 4),
                      "event_ms": round(statistics.median(evs), 4),
                      "gap_us": round((statistics.median(walls) - statistics.median(evs)) * 1e3, 1),
                      "walls": [round(x, 4) for x in walls]}))


if __name__ == "__main__":
    main()
