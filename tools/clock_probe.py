"""Is the rollout's fast/slow spread a clock (power-management) state?  Runs the bench's K = 20
rollout (2^20 envs, L = 36, int32 trajectory, RolloutPlan) back to back for a few seconds,
timing every launch with HIP events, while a thread samples `rocm-smi --showmetrics` (read
only: current gfx / memory / fabric / SoC clocks, activity, power).  Prints one JSON object:
per-launch ms with host timestamps, and the metric samples with theirs.

    python tools/clock_probe.py [--seconds 4] [--idle 1.0]
"""
import argparse
import json
import os
import re
import subprocess
import sys
import threading
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "ac-solver-caltech_amd"))
from bench import ms_starts  # noqa: E402
from acx import ops  # noqa: E402

KEYS = ("current_gfxclk", "current_uclk", "current_fclk", "current_socclk", "average_gfx_activity",
        "average_umc_activity", "current_socket_power", "average_socket_power", "temperature_hbm",
        "temperature_hotspot", "throttle_status", "indep_throttle_status")


def sample(raw=False):
    try:
        out = subprocess.run(["rocm-smi", "--showmetrics"], capture_output=True, text=True, timeout=20).stdout
    except Exception as e:  # noqa: BLE001
        return {"error": str(e)}
    rec = {}
    if raw:
        rec["raw"] = out
        try:
            rec["static"] = subprocess.run(
                ["rocm-smi", "--showmemorypartition", "--showcomputepartition", "--showperflevel", "--showmaxpower",
                 "--showclkfrq", "--showmemvendor", "--showvbios", "--showdriverversion"],
                capture_output=True, text=True, timeout=30).stdout
        except Exception as e:  # noqa: BLE001
            rec["static"] = str(e)
    for line in out.splitlines():
        for k in KEYS:
            m = re.search(rf"\b{k}\b[^:]*:\s*(.+)$", line)
            if m and k not in rec:
                rec[k] = m.group(1).strip()[:200]
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=4.0)
    ap.add_argument("--idle", type=float, default=1.0)
    a = ap.parse_args()
    t_origin = time.perf_counter()
    samples = [{"t": 0.0, "phase": "before_alloc", **sample(raw=True)}]
    B, L, H, K, dev = 1 << 20, 36, 200, 20, torch.device("cuda:0")
    starts = torch.as_tensor(ms_starts(L, B)).to(dev)
    state = starts.clone()
    cnt = torch.zeros(B, dtype=torch.int32, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    acts = torch.randint(0, 12, (K, B), dtype=torch.int32, device=dev, generator=g)
    obs = torch.zeros((K, B, 2 * L), dtype=torch.int32, device=dev)
    rew = torch.zeros((K, B), dtype=torch.int32, device=dev)
    dn = torch.zeros((K, B), dtype=torch.uint8, device=dev)
    tr = torch.zeros((K, B), dtype=torch.uint8, device=dev)
    err = torch.zeros(B, dtype=torch.uint8, device=dev)
    ec = torch.zeros(1, dtype=torch.int32, device=dev)
    plan = ops.RolloutPlan(state, starts, cnt, T=K, horizon=H, obs_traj=obs, reward_traj=rew, done_traj=dn,
                           trunc_traj=tr, err=err, err_count=ec)
    plan(acts)
    torch.cuda.synchronize()
    time.sleep(a.idle)
    samples.append({"t": time.perf_counter() - t_origin, "phase": "idle_after_alloc", **sample()})
    stop = threading.Event()

    def poll():
        while not stop.is_set():
            s = sample()
            samples.append({"t": time.perf_counter() - t_origin, "phase": "busy", **s})

    th = threading.Thread(target=poll, daemon=True)
    th.start()
    launches = []
    t_end = time.perf_counter() + a.seconds
    while time.perf_counter() < t_end:
        evs = []
        t_host = time.perf_counter() - t_origin
        for _ in range(20):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            plan(acts)
            e1.record()
            evs.append((e0, e1))
        torch.cuda.synchronize()
        launches.append({"t": t_host, "ms": [round(e0.elapsed_time(e1), 4) for e0, e1 in evs]})
    stop.set()
    th.join(timeout=30)
    time.sleep(a.idle)
    samples.append({"t": time.perf_counter() - t_origin, "phase": "idle_after", **sample()})
    # one more short batch after the idle gap: does the first launch after idling run slower?
    evs = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        plan(acts)
        e1.record()
        evs.append((e0, e1))
    torch.cuda.synchronize()
    after_idle = [round(e0.elapsed_time(e1), 4) for e0, e1 in evs]
    allms = [m for b in launches for m in b["ms"]]
    allms.sort()
    print(json.dumps({"n_launches": len(allms), "median_ms": allms[len(allms) // 2], "min_ms": allms[0],
                      "max_ms": allms[-1], "after_idle_ms": after_idle, "batches": launches, "samples": samples,
                      "env_errors": int(ec.item())}))


if __name__ == "__main__":
    main()
