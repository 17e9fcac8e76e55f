#!/usr/bin/env python3
"""Benchmark: env-steps/sec at batch 2^20, max_relator_length 36 (BASELINE.json metric).

Workload (BASELINE.json configs[2]): PPO rollout collection -- 2^20 envs per GPU,
L = 36, env horizon 200, Miller-Schupp starting states (env i starts at presentation
i mod 1190 of all_presentations.txt), uniform random move ids pre-generated on the device
(torch.Generator, seed 0 + rank), same-step autoreset.  One bench "step" = one env step of
the whole batch; the K timed steps are acx_rollout launches of <= 200 steps (one for the
default K = 200; a larger K reuses the same buffers, as a PPO loop does) that write the full
(K, B, 2L) int32 observation trajectory plus reward/done/truncated per step.  Inputs are
resident in HBM before the timed region.

Also measured (reported under "variants"): the per-call acx_step API (one launch per step,
state read+written in HBM each step) on the same batch.

Multi-GPU: one process per GPU (torchrun), envs sharded by index (weak scaling: 2^20
envs per rank); no collective on the data path, a barrier + max-over-ranks of the timed
region only.

CPU baseline (rank 0, N = 1): oracle/np_port.py -- a numpy restatement with the reference's
per-env ACEnv.step call pattern -- one process per host core (bounded at 16), 64 envs each,
~10 s, same starting states and action stream.  Run before the GPU is touched.
"""

from __future__ import annotations

import argparse
import contextlib
import io
import json
import os
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.join(REPO, "ac-solver-caltech_amd")
sys.path.insert(0, PKG_ROOT)
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, MI355X_MICROARCH.md "Chip-level parameters"


def nw_for(L: int) -> int:
    """32-bit words per packed relator in the kernel instantiation (csrc/acx_kernels.hip)."""
    return 1 if L <= 16 else 2 if L <= 32 else 3 if L <= 48 else 4 if L <= 64 else 8


def ms_starts(L: int, B: int, offset: int = 0) -> np.ndarray:
    ms = np.load(os.path.join(PKG_ROOT, "acx", "data", "all_presentations.npy"))
    idx = (np.arange(B) + offset) % len(ms)
    src = ms[idx]
    out = np.zeros((B, 2 * L), np.int32)
    for h in range(2):
        half = src[:, h * 18 : (h + 1) * 18]
        out[:, h * L : h * L + 18] = half
    return out


def cpu_baseline(L: int, horizon: int, seconds: float, max_procs: int = 16):
    """numpy reference-structured port, one process per core, bounded sample."""
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    procs_n = max(1, min(cores, max_procs))
    code = (
        "import sys,json,numpy as np; sys.path.insert(0,%r); sys.path.insert(0,%r);"
        "from bench import ms_starts; from oracle import np_port;"
        "r=int(sys.argv[1]); s=ms_starts(%d,64,offset=64*r).astype(np.int64);"
        "a=np.random.default_rng(r).integers(0,12,size=(4096,64));"
        "n,el=np_port.run_sample(s,a,%d,%f); print(json.dumps([n,el]))"
    ) % (REPO, PKG_ROOT, L, horizon, seconds)
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
    ps = [subprocess.Popen([sys.executable, "-c", code, str(r)], stdout=subprocess.PIPE, env=env)
          for r in range(procs_n)]
    total = 0.0
    for p in ps:
        out, _ = p.communicate(timeout=seconds * 10 + 120)
        n, el = json.loads(out.decode().strip().splitlines()[-1])
        total += n / el
    return {
        "value": total,
        "unit": "env-steps/s",
        "cores": procs_n,
        "kind": "port",
        "sample": f"oracle/np_port.py ACEnv.step restatement, {procs_n} procs x 64 envs x {seconds:.0f}s, "
                  f"L={L}, horizon {horizon}, Miller-Schupp starts, uniform actions",
    }


def cpu_baseline_c(L: int, horizon: int, seconds: float):
    """C oracle (oracle/acx_oracle.c), one core, batch of 65536 envs (second CPU number)."""
    from oracle import oracle as O

    B = 65536
    starts = ms_starts(L, B)
    state = starts.copy()
    cnt = np.zeros(B, np.int32)
    rng = np.random.default_rng(0)
    steps = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        O.env_step(state, rng.integers(0, 12, size=B).astype(np.int32), L, horizon, cnt, reset_state=starts)
        steps += B
    el = time.perf_counter() - t0
    return {"value": steps / el, "unit": "env-steps/s", "cores": 1, "kind": "port",
            "sample": f"oracle/acx_oracle.c env_step, 1 core, B=65536, {el:.1f}s"}


def cpu_baseline_c_all(L: int, horizon: int, seconds: float, max_procs: int = 16):
    """C oracle on every host core (one process each, <= 16, 16384 envs each): the strongest
    CPU number (SURVEY 8d asks for the C++ restatement on one core and on all cores)."""
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    procs_n = max(1, min(cores, max_procs))
    code = (
        "import sys,json,time,numpy as np; sys.path.insert(0,%r); sys.path.insert(0,%r);"
        "from bench import ms_starts; from oracle import oracle as O;"
        "r=int(sys.argv[1]); B=16384; s0=ms_starts(%d,B,offset=B*r); st=s0.copy(); c=np.zeros(B,np.int32);"
        "rng=np.random.default_rng(r); n=0; t0=time.perf_counter()\n"
        "while time.perf_counter()-t0<%f:\n"
        "  O.env_step(st,rng.integers(0,12,size=B).astype(np.int32),%d,%d,c,reset_state=s0); n+=B\n"
        "print(json.dumps([n,time.perf_counter()-t0]))"
    ) % (REPO, PKG_ROOT, L, seconds, L, horizon)
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
    ps = [subprocess.Popen([sys.executable, "-c", code, str(r)], stdout=subprocess.PIPE, env=env)
          for r in range(procs_n)]
    total = 0.0
    for p in ps:
        out, _ = p.communicate(timeout=seconds * 10 + 120)
        n, el = json.loads(out.decode().strip().splitlines()[-1])
        total += n / el
    return {"value": total, "unit": "env-steps/s", "cores": procs_n, "kind": "port",
            "sample": f"oracle/acx_oracle.c env_step, {procs_n} procs x 16384 envs x {seconds:.0f}s"}


def dist_setup(local_rank: int, world: int, backend: str = "nccl", force: bool = False):
    """One process per GPU (torchrun's LOCAL_RANK / WORLD_SIZE / MASTER_*): select this rank's
    GPU and, for world > 1 (or `force`, a one-rank group: tests/test_gpu_sbfs.py runs the RCCL
    path that way on one GPU), join the process group -- "nccl" is RCCL over xGMI, bound to the
    rank's device; "gloo" rehearses N ranks on one GPU.  Returns the rank's device."""
    import torch
    import torch.distributed as dist

    gpu = local_rank if backend == "nccl" else local_rank % torch.cuda.device_count()
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if world > 1 or force:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    return dev


def synced_max(value: float, dev) -> float:
    """max over the ranks of a host float (the timed region's wall time): an RCCL all_reduce of a
    device scalar; the value itself in a single process without a process group."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return value
    t = torch.tensor([value], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier() -> None:
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        dist.barrier()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=1 << 20, help="envs per GPU")
    ap.add_argument("--L", type=int, default=36)
    ap.add_argument("--horizon", type=int, default=200)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-step-api", action="store_true")
    ap.add_argument("--no-learner", action="store_true")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-bfs", action="store_true")
    ap.add_argument("--no-desync", action="store_true")
    ap.add_argument("--no-obs8", action="store_true")
    ap.add_argument("--bfs-timeout", type=float, default=180.0,
                    help="world > 1: seconds the sharded-BFS variant may take before the line is printed without it")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    L, B, K, W, H = args.L, args.batch, args.steps, args.warmup, args.horizon

    cpu = None
    cpu_c = None
    cpu_c_all = None
    if rank == 0 and world == 1 and not args.no_cpu:
        # before anything touches the GPU
        cpu = cpu_baseline(L, H, args.cpu_seconds)
        cpu_c = cpu_baseline_c(L, H, min(5.0, args.cpu_seconds))
        cpu_c_all = cpu_baseline_c_all(L, H, min(5.0, args.cpu_seconds))

    import torch
    import torch.distributed as dist

    backend = os.environ.get("ACX_DIST_BACKEND", "nccl")  # "gloo": rehearse N ranks on one GPU
    dev = dist_setup(local_rank, world, backend)

    import acx
    from acx import ops

    starts = torch.as_tensor(ms_starts(L, B, offset=rank * B)).to(dev)
    state = starts.clone()
    count = torch.zeros(B, dtype=torch.int32, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(0 + rank)
    # one launch's obs trajectory is T*B*8L bytes (60.4 GB at T = 200, L = 36); a K beyond
    # the PPO horizon chunk runs as consecutive launches of <= T_CHUNK steps that reuse the
    # same buffers (a PPO loop reuses its rollout storage the same way)
    T_CHUNK = max(1, min(200, (160 << 30) // max(1, B * (8 * L + 10))))
    T_buf = min(max(K, W), T_CHUNK)
    actions = torch.randint(0, 12, (W + K, B), dtype=torch.int32, device=dev, generator=g)
    obs = torch.empty((T_buf, B, 2 * L), dtype=torch.int32, device=dev)
    rew = torch.empty((T_buf, B), dtype=torch.int32, device=dev)
    done = torch.empty((T_buf, B), dtype=torch.uint8, device=dev)
    trunc = torch.empty((T_buf, B), dtype=torch.uint8, device=dev)
    err = torch.zeros(B, dtype=torch.uint8, device=dev)
    err_count = torch.zeros(1, dtype=torch.int32, device=dev)
    # a PPO loop reuses its rollout buffers; touch them once (untimed) so the timed region
    # does not pay first-touch page mapping of a fresh 60 GB allocation
    for buf in (obs, rew, done, trunc):
        buf.zero_()

    # the launches go through ops.RolloutPlan (checks and pointers resolved once per chunk
    # length, as a PPO loop reusing its buffers would); same kernels and results as ops.rollout
    plans = {}

    def plan(n):
        if n not in plans:
            plans[n] = ops.RolloutPlan(state, starts, count, T=n, horizon=H, cyclical=True, obs_traj=obs[:n],
                                       reward_traj=rew[:n], done_traj=done[:n], trunc_traj=trunc[:n], err=err,
                                       err_count=err_count)
        return plans[n]

    def roll(a, T):
        for t0 in range(0, T, T_buf):
            t1 = min(T, t0 + T_buf)
            plan(t1 - t0)(a[t0:t1])

    plan(min(K, T_buf)), plan(K % T_buf or T_buf)  # built before the timed region

    # warmup (W env steps, untimed)
    if W > 0:
        roll(actions[:W], W)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    roll(actions[W : W + K], K)
    t_launch = time.perf_counter() - t0
    ev1.record()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kernel_s = ev0.elapsed_time(ev1) / 1e3
    elapsed = synced_max(elapsed, dev)
    n_err = int(err_count.item())  # the headline rollout's env errors (warmup + timed)

    # algorithmic bytes of the rollout launch (DESIGN.md "Roofline"): per env-step action 4 B
    # + obs 8L B + reward 4 + done 1 + truncated 1; per env per launch state in/out 2*8L,
    # step count in/out 8, err 1; plus the starting state (8L) of every env that resets
    step_bytes = 4 + 8 * L + 4 + 1 + 1
    n_launch = -(-K // T_buf)

    def count_resets(T):
        # resets of the last launch = done | truncated over its steps (both never hold together
        # in a way that matters: a reset reads one row either way)
        if T > T_buf:
            return None
        return int((done[:T] | trunc[:T]).sum().item())

    def rollout_bytes(n_resets):
        return K * B * step_bytes + n_launch * B * (16 * L + 8 + 1) + (n_resets or 0) * 8 * L

    resets = count_resets(K)
    launch_bytes = rollout_bytes(resets)
    achieved = launch_bytes / kernel_s / 1e9

    variants = {}

    def desync_variant(start_rows, count0, what):
        # the rollout with the episodes out of phase (step_count[i] = i mod H): ~B/H envs reset
        # on every step, scattered over the waves -- the steady state of a PPO rollout, which
        # the headline's synchronised counts (all 0 at the start) never show in K < H steps
        st = start_rows.clone()
        cnt = count0.clone()
        err_count.zero_()

        def go(a, T):
            for t0 in range(0, T, T_buf):
                t1 = min(T, t0 + T_buf)
                ops.rollout(st, a[t0:t1], start_rows, cnt, horizon=H, cyclical=True, obs_traj=obs[: t1 - t0],
                            reward_traj=rew[: t1 - t0], done_traj=done[: t1 - t0], trunc_traj=trunc[: t1 - t0],
                            err=err, err_count=err_count)

        if W > 0:
            go(actions[:W], W)
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        go(actions[W : W + K], K)
        e1.record()
        torch.cuda.synchronize()
        s_d = e0.elapsed_time(e1) / 1e3
        nres = count_resets(K)
        nb = rollout_bytes(nres)
        return {"value": B * K / s_d, "unit": "env-steps/s", "kernel_ms": s_d * 1e3, "ms_per_step": s_d / K * 1e3,
                "resets_per_step": None if nres is None else nres / K, "env_errors": int(err_count.item()),
                "workload": what,
                "roofline": {"bound": "hbm", "achieved": nb / s_d / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": nb / s_d / 1e9 / HBM_PEAK_GBS, "launch_bytes": nb}}

    if not args.no_obs8:
        # the headline rollout (same starts, counts from 0, same actions) with the observation
        # trajectory in the reference's observation dtype, int8 (ac_env.py:64-70: Box(int8); the
        # observations SyncVectorEnv returns): 2L bytes per env-step instead of 8L
        obs8 = torch.zeros((T_buf, B, 2 * L), dtype=torch.int8, device=dev)
        st8, cnt8 = starts.clone(), torch.zeros(B, dtype=torch.int32, device=dev)
        err_count.zero_()

        def go8(a, T):
            for t0 in range(0, T, T_buf):
                t1 = min(T, t0 + T_buf)
                ops.rollout(st8, a[t0:t1], starts, cnt8, horizon=H, cyclical=True, obs_traj=obs8[: t1 - t0],
                            reward_traj=rew[: t1 - t0], done_traj=done[: t1 - t0], trunc_traj=trunc[: t1 - t0],
                            err=err, err_count=err_count)

        if W > 0:
            go8(actions[:W], W)
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        go8(actions[W : W + K], K)
        e1.record()
        torch.cuda.synchronize()
        s8 = e0.elapsed_time(e1) / 1e3
        nres = count_resets(K)
        nb8 = rollout_bytes(nres) - K * B * 6 * L  # obs 2L instead of 8L bytes per env-step
        variants["rollout_obs_int8"] = {
            "value": B * K / s8, "unit": "env-steps/s", "kernel_ms": s8 * 1e3, "ms_per_step": s8 / K * 1e3,
            "env_errors": int(err_count.item()),
            "workload": "the headline rollout writing the (K,B,2L) observation trajectory as int8 (the reference's "
                        "observation_space dtype) instead of int32",
            "roofline": {"bound": "hbm", "achieved": nb8 / s8 / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": nb8 / s8 / 1e9 / HBM_PEAK_GBS, "launch_bytes": nb8,
                         "bytes_per_env_step": step_bytes - 6 * L}}
        del obs8, st8, cnt8

    if not args.no_desync:
        desync = torch.arange(B, dtype=torch.int32, device=dev) % H
        variants["rollout_desync"] = desync_variant(
            starts, desync, "the headline rollout with step_count[i] = i mod H (Miller-Schupp starts): about B/H "
                            "truncations per step, scattered over the waves")
        triv = np.zeros((8, 2 * L), np.int32)
        for r, (a0, a1) in enumerate([(1, 2), (1, -2), (-1, 2), (-1, -2), (2, 1), (2, -1), (-2, 1), (-2, -1)]):
            triv[r, 0], triv[r, L] = a0, a1
        tstarts = torch.as_tensor(triv[np.arange(B) % 8]).to(dev)
        variants["rollout_done_heavy"] = desync_variant(
            tstarts, desync, "done-heavy: every env starts at one of the 8 trivial presentations "
                             "(generate_trivial_states, utils.py:91-114) with step_count[i] = i mod H, so dones "
                             "and resets fire on a large share of env-steps")
        del tstarts, desync
    chg_rate = None  # changed relators per env-step of the in-place step (step_api variant)
    if not args.no_step_api:
        # per-call acx_step API: one launch per env step, state in/out of HBM each step
        rew1 = torch.empty(B, dtype=torch.int32, device=dev)
        dn1 = torch.empty(B, dtype=torch.uint8, device=dev)
        tr1 = torch.empty(B, dtype=torch.uint8, device=dev)
        lens1 = torch.empty((B, 2), dtype=torch.int32, device=dev)
        st1 = starts.clone()
        cnt1 = torch.zeros(B, dtype=torch.int32, device=dev)

        def step(a):
            ops.step(st1, a, state_out=st1, reset_state=starts, step_count=cnt1, horizon=H, cyclical=True,
                     reward=rew1, done=dn1, truncated=tr1, lengths=lens1, err=err, err_count=err_count)

        err_count.zero_()
        for t in range(W):
            step(actions[t])
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for t in range(K):
            step(actions[W + t])
        e1.record()
        torch.cuda.synchronize()
        s_api = e0.elapsed_time(e1) / 1e3
        n_err_api = int(err_count.item())
        # The in-place step writes back only the relators that changed (gated moves, no-op
        # cyclic conjugations and failed envs leave their rows as they are in HBM), so the bytes
        # it must move depend on the walk: measured off the clock over the next 8 steps of the
        # same walk as the mean number of changed relators per env-step.
        chg = 0.0
        for t in range(8):
            before = st1.clone()
            step(actions[(W + K + t) % actions.shape[0]])
            chg += float(((before.view(B, 2, L) != st1.view(B, 2, L)).any(2)).sum().item()) / B
            del before
        chg /= 8
        chg_rate = chg
        # per env-step: state in 8L + action 4 + count in 4 + changed relators x 4L + lengths 8 +
        # reward 4 + done 1 + truncated 1 + count out 4 + err 1; full rows: state out 8L
        sb_full = 16 * L + 27
        sb = 8 * L + 27 + 4 * L * chg
        variants["step_api"] = {
            "value": world * B * K / s_api if world == 1 else None,
            "unit": "env-steps/s",
            "ms_per_step": s_api / K * 1e3,
            "roofline": {"bound": "hbm", "achieved": B * sb / (s_api / K) / 1e9, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": B * sb / (s_api / K) / 1e9 / HBM_PEAK_GBS,
                         "bytes_per_env_step": sb, "changed_relators_per_env_step": chg,
                         "bytes_per_env_step_full_rows": sb_full,
                         "frac_on_full_row_bytes": B * sb_full / (s_api / K) / 1e9 / HBM_PEAK_GBS},
            "env_errors": n_err_api,
        }

        # the same K per-call steps captured once into a hipGraph (torch.cuda.CUDAGraph over
        # the ctypes launches on the capture stream) and replayed: no per-launch host cost
        if not args.no_graph:
            gs = torch.cuda.Stream(device=dev)
            gs.wait_stream(torch.cuda.current_stream(dev))
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.stream(gs):
                with torch.cuda.graph(graph, stream=gs):
                    for t in range(K):
                        step(actions[W + t])
            torch.cuda.synchronize()
            graph.replay()  # warm
            torch.cuda.synchronize()
            e0.record()
            graph.replay()
            e1.record()
            torch.cuda.synchronize()
            s_g = e0.elapsed_time(e1) / 1e3
            variants["step_api_hipgraph"] = {
                "value": B * K / s_g if world == 1 else None, "unit": "env-steps/s", "ms_per_step": s_g / K * 1e3,
                "roofline": {"bound": "hbm", "achieved": B * sb / (s_g / K) / 1e9, "peak": HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": B * sb / (s_g / K) / 1e9 / HBM_PEAK_GBS,
                             "bytes_per_env_step": sb, "bytes_per_env_step_full_rows": sb_full},
            }
            del graph

    if not args.no_learner and world == 1:
        # PPO plumbing (acx.agents.LearnerEnv): per step one acx_step_learner (int64 policy
        # actions in, float32 obs straight into the learner's (T+1,B,2L) buffer, float32
        # reward/done, episode move history) + one acx_curriculum_assign
        from acx.agents import LearnerEnv
        KL = min(K, 50)
        lenv = LearnerEnv(np.concatenate([ms_starts(L, B), ms_starts(L, 4096, offset=B)]), B, horizon_length=H,
                          device=dev)
        lobs = torch.empty((KL + 1, B, 2 * L), dtype=torch.float32, device=dev)
        lrew = torch.empty((KL, B), dtype=torch.float32, device=dev)
        ldone = torch.empty((KL, B), dtype=torch.float32, device=dev)
        la = actions[W : W + KL].to(torch.int64)
        lobs.zero_()
        lenv.step(la[0], obs_out=lobs[1], reward_out=lrew[0], done_out=ldone[0])
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for t in range(KL):
            lenv.step(la[t], obs_out=lobs[t + 1], reward_out=lrew[t], done_out=ldone[t])
        e1.record()
        torch.cuda.synchronize()
        s_l = e0.elapsed_time(e1) / 1e3
        # per env-step: state in/out 16L + action 8 + count in/out 8 + obs f32 8L + reward f32 4
        # + done f32 4 + done/trunc u8 2 + history 1 + episode_len 4 + err 1 + curriculum
        # (done/trunc re-read 2, needs_host 1)
        # The state store is in place (changed relators only, see step_api): the same walk
        # distribution as the step_api variant (Miller-Schupp starts, uniform moves, horizon H),
        # so its measured changed-relator rate prices the state write-back.
        lb_full = 24 * L + 35
        lb = lb_full if chg_rate is None else lb_full - 8 * L + 4 * L * chg_rate
        variants["learner_step"] = {
            "value": B * KL / s_l, "unit": "env-steps/s", "steps": KL, "ms_per_step": s_l / KL * 1e3,
            "roofline": {"bound": "hbm", "achieved": B * lb / (s_l / KL) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": B * lb / (s_l / KL) / 1e9 / HBM_PEAK_GBS, "bytes_per_env_step": lb,
                         "bytes_per_env_step_full_rows": lb_full,
                         "frac_on_full_row_bytes": B * lb_full / (s_l / KL) / 1e9 / HBM_PEAK_GBS},
        }
        del lobs, lrew, ldone, lenv

    def sharded_bfs_variant():
        # BASELINE configs[3] on the owner-partitioned BFS (csrc/acx_sbfs.hip): AK(3), L = 36, to
        # 10^7 nodes; node store + visited set sharded over the ranks by key owner, per-chunk RCCL
        # all_gather / all_to_all / all_reduce (world 1: the exchanges are local copies)
        from acx.envs.utils import convert_relators_to_presentation
        from acx.search import _sharded_bfs as SB
        ak3 = convert_relators_to_presentation([1, 1, 1, -2, -2, -2, -2], [1, 2, 1, -2, -1, -2], 36)
        nb = 10 ** 7
        with contextlib.redirect_stdout(io.StringIO()):
            SB.sharded_bfs(ak3, nb, device=dev)  # warmup: workspace allocation
        best = None
        for _ in range(3):
            barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            with contextlib.redirect_stdout(io.StringIO()):
                res = SB.sharded_bfs(ak3, nb, device=dev)
            torch.cuda.synchronize()
            el = synced_max(time.perf_counter() - t0, dev)
            best = el if best is None else min(best, el)
        st = SB.LAST_STATS
        return {
            "value": st["nodes"] / best, "unit": "BFS nodes/s", "wall_ms": best * 1e3, "nodes": st["nodes"],
            "parents_expanded": st["parents"], "chunks": st["chunks"], "result": list(res) if res[0] else [False, None],
            "workload": "BASELINE configs[3]: bfs from AK(3), L=36, cyclical=False, to 10^7 nodes; node store and "
                        f"visited set partitioned by key owner over {world} rank(s), "
                        f"{'RCCL' if backend == 'nccl' else backend} exchanges per chunk",
        }

    # HBM traffic per launch from rocprofv3 PMC (FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md
    # "HBM"), measured by profile_cmd.sh on this same command and committed under profiles/;
    # used only when that profile's workload matches this run's
    # (the newest committed profile of this workload at this K; profile_cmd.sh profiles the
    # driver's own command, bench.py --steps 20 --warmup 5, and the K = 200 default)
    # A profile of the same (B, L, K) gives the launch's measured bytes directly; one of another K
    # is carried over as its measured/algorithmic ratio (the launch's bytes are the same per-step
    # and per-launch terms at any K, so the ratio is K-independent) and labelled as scaled.
    traffic, traffic_src = None, None
    cands = []
    for tag in ("r03v_k20", "r03v", "r03m_k20", "r03m", "r02o_k20", "r02o", "r02h_k20", "r02h", "r02_k20", "r02", "r01"):
        prof = os.path.join(REPO, "profiles", tag.split("_")[0][:3], f"{tag}_summary.json")
        if not os.path.exists(prof):
            continue
        with open(prof) as f:
            ps = json.load(f)
        pc = ps.get("bench_line", {}).get("config", {})
        td = ps.get("rollout_timed_dispatch") or {}
        if pc.get("envs_per_gpu") == B and pc.get("max_relator_length") == L and td.get("pmc_hbm_bytes"):
            cands.append((ps["bench_line"].get("steps") != K, tag, ps["bench_line"].get("steps"), td))
    if cands:
        scaled, tag, kp, td = min(cands, key=lambda c: c[0])
        where = f"profiles/{tag.split('_')[0][:3]}/{tag}_summary.json: rocprofv3 --pmc FETCH_SIZE (x2) + --pmc WRITE_SIZE"
        if not scaled:
            traffic, traffic_src = td["pmc_hbm_bytes"], f"{where} of this command (K={K})"
        else:
            ratio = td["pmc_hbm_bytes"] / td["algorithmic_bytes"]
            traffic = launch_bytes * ratio
            traffic_src = (f"{where} at K={kp}: measured/algorithmic = {ratio:.4f}, applied to this launch's "
                           "algorithmic bytes")

    value = world * B * K / elapsed
    line = {
        "metric": "env-steps/sec at batch 2^20, max_relator_len 36; 1/2/4/8 MI355X",
        "value": value,
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": K,
        "warmup": W,
        "ms_per_step": elapsed / K * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic: Miller-Schupp starting states (all_presentations.txt, env i -> i mod 1190), "
                "uniform random move ids (torch.Generator seed 0+rank)",
        "config": {
            "workload": (f"PPO rollout collection (BASELINE configs[2]): {B} envs/GPU, L={L}, horizon {H}, "
                         "cyclical=True, same-step autoreset, full (K,B,2L) int32 obs trajectory; "
                         f"acx_rollout launches of <= {T_buf} steps ({n_launch} for K={K})"),
            "global_batch": world * B,
            "envs_per_gpu": B,
            "max_relator_length": L,
            "horizon": H,
            "parallelism": f"env-index shards x{world}, no data-path collective",
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "traffic_source": traffic_src,
            "kernel": ("acx::pack_actions_kernel + " if plan(min(K, T_buf)).packs else "")
            + f"acx::rollout_kernel<{nw_for(L)},{L if L in (36, 128) else 0},4,1>",
            "bytes_per_env_step": step_bytes,
            "launch_bytes": launch_bytes,
            "resets_in_launch": resets,
            "launches": n_launch,
            "kernel_ms": kernel_s * 1e3,
            "host_launch_ms": t_launch * 1e3,
        },
        "cpu_baseline": cpu,
        "cpu_baseline_c_oracle": cpu_c,
        "cpu_baseline_c_oracle_all_cores": cpu_c_all,
        "variants": variants,
        "env_errors": n_err,
    }
    if not args.no_bfs:
        # last, behind a watchdog: the one variant with collectives on its data path.  If its RCCL
        # exchanges at world > 1 ever stalled, every rank's watchdog prints the line (rank 0) with
        # the variant marked and exits, so a hang there cannot cost the headline line
        import threading

        from acx.search import _sharded_bfs as SB
        variants["sharded_bfs"] = {"error": f"timeout after {args.bfs_timeout:.0f} s"}
        timed_out_line = json.dumps(line)

        def on_timeout():
            if rank == 0:  # the variant may be inside redirect_stdout: write to the real stdout
                sys.__stdout__.write(timed_out_line + "\n")
                sys.__stdout__.flush()
            os._exit(0)

        dog = threading.Timer(args.bfs_timeout, on_timeout) if world > 1 else None
        if dog is not None:
            dog.daemon = True
            dog.start()
        try:  # a variant: its failure (the same on every rank) must not cost the headline line
            variants["sharded_bfs"] = sharded_bfs_variant()
        except Exception as e:  # noqa: BLE001
            variants["sharded_bfs"] = {"error": repr(e)[:300]}
        if dog is not None:
            dog.cancel()
        SB.release_workspaces()

    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
