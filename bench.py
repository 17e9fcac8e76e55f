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

`--workload step` makes the per-call step API (one launch per env step, random actions,
in-place state, autoreset) the headline instead -- the call VecACEnv.step makes: at L = 128
acx_step_lengths (the rows' relator lengths in and out, only the chunks inside the letters read
and written), otherwise acx_step; the other call on the same walk is a variant.  BASELINE
configs[4] ("random-action stepping", L = 128, 2^20 envs per GPU over 8 GPUs) is

    python bench.py --gpus 8 --workload step --L 128 --batch 1048576

Also measured (reported under "variants"): the rollout with an int8 trajectory and with scattered
resets, the per-call step API (+ hipGraph), the PPO learner step, config 4's searches (device BFS,
expansion kernel, host-dedup BFS, owner-partitioned BFS).

Multi-GPU: one process per GPU, envs sharded by index (weak scaling: B envs per rank, or with
`--global-batch G` strong scaling: G / N envs per rank, "scaling": "strong"); no
collective on the data path, a barrier + max-over-ranks of every timed region only.  Either
torchrun starts the ranks (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in the environment), or
`--gpus N > 1` without them makes this process a launcher that starts N rank processes of this
script itself (children, never an exec) and exits with their status.  Every rank checks that the
process group it joined has exactly --gpus ranks.

CPU baseline (every N): oracle/np_port.py -- a numpy restatement with the reference's per-env
ACEnv.step call pattern -- one process per host core (bounded at 16), 64 envs each, ~10 s, same
starting states and action stream, plus the C oracle on one core and on every core.  Measured
once per run before any rank touches the GPU: by the launcher before it starts the ranks (`--gpus
N` on its own; handed to rank 0 through a JSON file named in ACX_BENCH_CPU_JSON), or by rank 0
before it joins the process group (torchrun), so every line -- N = 1, 2, 4, 8 -- carries it.

`--dry-run` exercises the launcher, the process group, the world-size check and the line's
per-rank fields with no GPU (gloo, a numpy pass per step instead of the kernels); its line says
so ("dry_run": true) and is never a measurement.
"""

from __future__ import annotations

import argparse
import contextlib
import io
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.join(REPO, "ac-solver-caltech_amd")
sys.path.insert(0, PKG_ROOT)
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, MI355X_MICROARCH.md "Chip-level parameters"
METRIC = "env-steps/sec at batch 2^20, max_relator_len 36; 1/2/4/8 MI355X"
EXIT_WORLD_MISMATCH = 2  # the process group does not have --gpus ranks
EXIT_BFS_STALL = 3       # the sharded-BFS variant's collectives stalled (line printed without it)


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


CPU_JSON_ENV = "ACX_BENCH_CPU_JSON"  # the launcher's CPU baselines, handed to rank 0


def cpu_baselines(args, where: str) -> dict:
    """the three CPU baselines of the line (numpy port on every core, C oracle on one core and on
    every core), measured here and now -- before anything in this process touches the GPU"""
    if args.no_cpu:
        return {}
    L, H = args.L, args.horizon
    out = {"cpu_baseline": cpu_baseline(L, H, args.cpu_seconds),
           "cpu_baseline_c_oracle": cpu_baseline_c(L, H, min(5.0, args.cpu_seconds)),
           "cpu_baseline_c_oracle_all_cores": cpu_baseline_c_all(L, H, min(5.0, args.cpu_seconds))}
    for v in out.values():
        v["measured"] = where
    return out


def cpu_for_rank(args, rank: int, world: int) -> dict:
    """this rank's CPU baselines for the line: rank 0 takes the launcher's (ACX_BENCH_CPU_JSON) or
    measures them itself before it joins the process group; other ranks report none"""
    if rank != 0 or args.no_cpu:
        return {}
    path = os.environ.get(CPU_JSON_ENV)
    if path:
        with open(path) as f:
            return json.load(f)
    return cpu_baselines(args, f"rank 0 of {world}, before the process group and the GPU" if world > 1
                         else "before the GPU is touched")


# ---------------------------------------------------------------------------------------------
# ranks: launcher, process group, cross-rank reductions
# ---------------------------------------------------------------------------------------------
def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n: int, argv: list, poll_s: float = 0.2) -> int:
    """`bench.py --gpus N` with no torchrun environment: start N rank processes of this script
    (RANK = LOCAL_RANK = r, WORLD_SIZE = N, MASTER_ADDR 127.0.0.1), before anything here touches
    the GPU.  The ranks are children (no exec).  Rank 0 prints the line.  When a rank exits
    non-zero, the others are stopped (their exact PIDs) and that status is returned."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                for q in live:
                    q.terminate()
        if live:
            time.sleep(poll_s)
    return rc


def dist_setup(local_rank: int, world: int, backend: str = "nccl", force: bool = False, cpu: bool = False):
    """One process per GPU (LOCAL_RANK / WORLD_SIZE / MASTER_* from torchrun or spawn_ranks):
    select this rank's GPU and, for world > 1 (or `force`, a one-rank group: tests/test_gpu_sbfs.py
    runs the RCCL path that way on one GPU), join the process group -- "nccl" is RCCL over xGMI,
    bound to the rank's device; "gloo" rehearses N ranks on one GPU (or, with `cpu`, on none).
    Returns the rank's device."""
    import torch
    import torch.distributed as dist

    if cpu:
        dev = torch.device("cpu")
    else:
        gpu = local_rank if backend == "nccl" else local_rank % torch.cuda.device_count()
        torch.cuda.set_device(gpu)
        dev = torch.device("cuda", gpu)
    if world > 1 or force:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    return dev


def _coll_device(dev):
    """where a small reduction tensor lives: the rank's GPU under RCCL, host memory otherwise"""
    import torch
    import torch.distributed as dist

    return dev if dist.get_backend() == "nccl" else torch.device("cpu")


def synced_max(value: float, dev) -> float:
    """max over the ranks of a host float (a timed region's wall time); the value itself in a
    single process without a process group."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return value
    t = torch.tensor([value], dtype=torch.float64, device=_coll_device(dev))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_rows(row, dev) -> list:
    """every rank's row of floats (all_gather), in rank order; [row] without a process group"""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return [list(map(float, row))]
    t = torch.tensor(list(map(float, row)), dtype=torch.float64, device=_coll_device(dev))
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [[float(v) for v in o.cpu().tolist()] for o in out]


def barrier() -> None:
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        dist.barrier()


def world_seen() -> int:
    import torch.distributed as dist

    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=1 << 20, help="envs per GPU (weak scaling)")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="strong scaling: this many envs in total, split evenly over the ranks (overrides --batch)")
    ap.add_argument("--L", type=int, default=36)
    ap.add_argument("--horizon", type=int, default=200)
    ap.add_argument("--workload", choices=("rollout", "step"), default="rollout",
                    help="headline: PPO rollout collection (configs[2]) or per-call random-action stepping "
                         "(configs[4])")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-step-api", action="store_true")
    ap.add_argument("--no-learner", action="store_true")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-bfs", action="store_true")
    ap.add_argument("--no-search", action="store_true", help="skip config 4's single-GPU search variants")
    ap.add_argument("--no-desync", action="store_true")
    ap.add_argument("--no-obs8", action="store_true")
    ap.add_argument("--no-config2", action="store_true", help="skip the configs[1] (65,536 envs) step variant")
    ap.add_argument("--bfs-timeout", type=float, default=60.0,
                    help="world > 1: seconds the sharded-BFS variant may take before the line is printed "
                         "without it (exit status 3)")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: launcher / process group / line plumbing only (gloo, numpy pass per step)")
    return ap.parse_args(argv)


def main():
    args = parse_args()
    if args.gpus < 1:
        sys.exit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # the CPU baselines on the host's cores before any rank starts (none of them is busy yet)
        tmp = None
        if not args.no_cpu:
            import tempfile

            fd, tmp = tempfile.mkstemp(prefix="acx_bench_cpu_", suffix=".json")
            with os.fdopen(fd, "w") as f:
                json.dump(cpu_baselines(args, f"launcher, before the {args.gpus} ranks started"), f)
            os.environ[CPU_JSON_ENV] = tmp
        try:
            rc = spawn_ranks(args.gpus, sys.argv[1:])
        finally:
            if tmp:
                os.unlink(tmp)
        sys.exit(rc)
    run_rank(args)


def _check_world(args, rank: int) -> int:
    seen = world_seen()
    if seen != args.gpus:
        sys.stderr.write(f"bench.py rank {rank}: process group has {seen} rank(s), --gpus {args.gpus}\n")
        sys.stderr.flush()
        sys.exit(EXIT_WORLD_MISMATCH)
    return seen


def per_rank_batch(args, world: int) -> tuple:
    """(envs per rank, "weak" | "strong"): --batch per rank, or --global-batch split over the ranks
    (weak scaling at 2^20 envs per GPU, strong scaling at a fixed total of 2^20)"""
    if not args.global_batch:
        return args.batch, "weak"
    if args.global_batch % (64 * world):
        sys.exit(f"--global-batch {args.global_batch} must be a multiple of 64 x {world} ranks")
    return args.global_batch // world, "strong"


def _per_rank_rows(rows):
    return [{"rank": i, "value": r[0], "kernel_ms": r[1], "frac": r[2], "wall_ms": r[3]} for i, r in enumerate(rows)]


def restore(snap, tensors) -> None:
    for x, y in zip(tensors, snap):
        x.copy_(y)


def replay_walk(step_fn, state, tensors, n: int, L: int, lens=None, finished=None, unread=None) -> dict:
    """What the n steps step_fn(0..n-1) will do from here, counted off the clock: they are run
    from a snapshot of `tensors` (every buffer the steps read and write; the kernels are
    deterministic, so the timed pass that follows takes this same walk) and the snapshot is put
    back.  Per env-step: "changed" relators (the in-place write-back's unit), with `lens` (the
    lengths-carrying step's (B, 2) lengths) the "live_read" / "live_written" bytes of 16-byte
    chunks, with `finished` ((done, truncated) uint8 tensors) the "finished" envs; `unread(t)`
    ((B, 2) bool, evaluated before step t) marks the relators that step leaves unread
    (acx_step_lengths_reduced's skipped relator)."""
    import torch

    snap = [t.clone() for t in tensors]
    B = state.shape[0]
    chg = rd = wr = fin = srd = swr = lrd = skp = 0.0
    if lens is not None:
        # byte offset of each relator in the (B, 2L) int32 state: the 64-B sectors its chunks touch
        rel0 = ((torch.arange(B, device=state.device, dtype=torch.int64) * 2 * L)[:, None]
                + torch.tensor([0, L], device=state.device, dtype=torch.int64)[None, :]) * 4

        def sectors(chunks):
            nb = chunks.to(torch.int64) * 16
            return torch.where(nb > 0, (rel0 + nb - 1) // 64 - rel0 // 64 + 1, torch.zeros_like(nb))
    for t in range(n):
        before = state.clone()
        n_before = lens.clone() if lens is not None else None
        keep = (~unread(t)).to(torch.int64) if unread is not None else 1
        if unread is not None:
            skp += float((1 - keep).sum().item())
        step_fn(t)
        ch = (before.view(B, 2, L) != state.view(B, 2, L)).any(2)
        chg += float(ch.sum().item())
        if lens is not None:
            c_old = (n_before.clamp(0, L) + 3) // 4
            c_new = (lens.clamp(0, L) + 3) // 4
            c_wr = torch.maximum(c_old, c_new)
            if L % 32 == 0:  # relators start on a 64-B sector: the kernel writes whole sectors (CodeTile::widen_lim)
                c_wr = torch.clamp((c_wr + 3) // 4 * 4, max=L // 4)
            rd += float((c_old * keep).sum().item()) * 16
            wr += float((c_wr * ch).sum().item()) * 16
            srd += float((sectors(c_old) * keep).sum().item()) * 64
            swr += float(sectors(torch.maximum(c_old, c_new) * ch).sum().item()) * 64
            # HBM reads whole 128-B lines (tools/line_probe.py: a read of 16, 32 or 64 B of a line
            # takes the whole line's time and one 128-B request); relators start on a line at
            # L % 32 == 0
            lrd += float((((c_old + 7) // 8) * keep).sum().item()) * 128
        if finished is not None:
            fin += float((finished[0] | finished[1]).sum().item())
        del before, n_before
    restore(snap, tensors)
    d = max(1, n) * B
    return {"changed": chg / d, "live_read": rd / d, "live_written": wr / d, "finished": fin / d,
            "sector_read": srd / d, "sector_written": swr / d, "line_read": lrd / d, "unread": skp / d}


def learner_buffers(lenv) -> list:
    """every device tensor a LearnerEnv step reads or writes (its own and its VecACEnv's)"""
    import torch

    out, seen = [], set()
    for obj in (lenv, lenv.vec):
        for v in vars(obj).values():
            if torch.is_tensor(v) and v.is_cuda and v.data_ptr() not in seen:
                seen.add(v.data_ptr())
                out.append(v)
    return out


def learner_bytes(L: int, changed: float, finished: float) -> float:
    """algorithmic bytes per env-step of acx_learner_step (one launch, curriculum fused): state
    read 8L, obs float32 8L, action int64 8, step count in/out 8, reward / done float32 8,
    done / truncated 2, move history 1 + its ring base read 4, episode length 4, err 1,
    needs_host 1; changed relators x 4L written in place; per finished env its next start row
    read 8L (curriculum or reset row), its reset row written 8L, curr_index 4 and the ring base of
    its next episode 4"""
    return 16 * L + 37 + 4 * L * changed + finished * (16 * L + 8)


def dry_run(args, rank: int, local_rank: int, world: int) -> None:
    """Launcher / process-group / line plumbing with no GPU: a numpy pass over this rank's
    (B, 2L) int32 shard per step stands in for the kernels (the CPU baselines are real)."""
    import torch.distributed as dist

    cpu = cpu_for_rank(args, rank, world)
    dev = dist_setup(local_rank, world, "gloo", cpu=True)
    seen = _check_world(args, rank)
    (B, scaling), L, K, W = per_rank_batch(args, seen), args.L, args.steps, args.warmup
    shard = ms_starts(L, B, offset=rank * B)
    acc = np.zeros(B, np.int64)

    def pass_(t):
        acc[:] += (shard != 0).sum(1) + t

    for t in range(W):
        pass_(t)
    barrier()
    t0 = time.perf_counter()
    for t in range(K):
        pass_(t)
    barrier()
    el = time.perf_counter() - t0
    elapsed = synced_max(el, dev)
    rows = gather_rows([B * K / el, el * 1e3, 0.0, el * 1e3], dev)
    line = {
        "metric": METRIC, "value": seen * B * K / elapsed, "unit": "env-steps/s", "n_gpus": seen, "steps": K,
        "warmup": W, "ms_per_step": elapsed / K * 1e3, "higher_is_better": True, "scaling": scaling,
        "vs_baseline": None, "dtype": "int32", "data": "dry run: no GPU work (launcher / process-group check)",
        "dry_run": True, "world_size_seen": seen, "per_rank": _per_rank_rows(rows),
        "config": {"workload": f"dry run ({args.workload})", "global_batch": seen * B, "envs_per_gpu": B,
                   "max_relator_length": L, "parallelism": f"env-index shards x{seen}, no data-path collective"},
        "cpu_baseline": cpu.get("cpu_baseline"), "cpu_baseline_c_oracle": cpu.get("cpu_baseline_c_oracle"),
        "cpu_baseline_c_oracle_all_cores": cpu.get("cpu_baseline_c_oracle_all_cores"),
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def run_rank(args):
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.dry_run:
        return dry_run(args, rank, local_rank, world)
    (B, scaling), L, K, W, H = per_rank_batch(args, world), args.L, args.steps, args.warmup, args.horizon

    # before anything touches the GPU (rank 0 at every N: the launcher's, or measured here)
    cpus = cpu_for_rank(args, rank, world)

    import torch
    import torch.distributed as dist

    backend = os.environ.get("ACX_DIST_BACKEND", "nccl")  # "gloo": rehearse N ranks on one GPU
    dev = dist_setup(local_rank, world, backend)
    seen = _check_world(args, rank)

    import acx  # noqa: F401
    from acx import ops

    def timed(fn):
        """(max-over-ranks wall seconds, this rank's HIP-event seconds on the current stream) of
        fn(), bracketed by barrier + synchronize on both sides"""
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        return synced_max(wall, dev), e0.elapsed_time(e1) / 1e3, wall

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
    rollout_head = args.workload == "rollout"
    err = torch.zeros(B, dtype=torch.uint8, device=dev)
    err_count = torch.zeros(1, dtype=torch.int32, device=dev)
    # the rollout variants (int8 trajectory, scattered resets) go with the rollout headline only
    do_obs8 = rollout_head and not args.no_obs8
    do_desync = rollout_head and not args.no_desync
    if rollout_head:
        obs = torch.empty((T_buf, B, 2 * L), dtype=torch.int32, device=dev)
        rew = torch.empty((T_buf, B), dtype=torch.int32, device=dev)
        done = torch.empty((T_buf, B), dtype=torch.uint8, device=dev)
        trunc = torch.empty((T_buf, B), dtype=torch.uint8, device=dev)
        # a PPO loop reuses its rollout buffers; touch them once (untimed) so the timed region
        # does not pay first-touch page mapping of a fresh 60 GB allocation
        for buf in (obs, rew, done, trunc):
            buf.zero_()
    n_launch = -(-K // T_buf)
    step_bytes = 4 + 8 * L + 4 + 1 + 1

    def count_resets(T):
        # resets of the last launch = done | truncated over its steps (a reset reads one row)
        if T > T_buf:
            return None
        return int((done[:T] | trunc[:T]).sum().item())

    def rollout_bytes(n_resets):
        # algorithmic bytes of the rollout launches (DESIGN.md "Roofline"): per env-step action 4 B
        # + obs 8L B + reward 4 + done 1 + truncated 1; per env per launch state in/out 2*8L,
        # step count in/out 8, err 1; plus the starting state (8L) of every env that resets
        return K * B * step_bytes + n_launch * B * (16 * L + 8 + 1) + (n_resets or 0) * 8 * L

    variants = {}
    head = {}  # the headline's timing and roofline

    if rollout_head:
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
        if W > 0:
            roll(actions[:W], W)  # warmup (W env steps, untimed)
        t_launch = [0.0]

        def go_head():
            t0 = time.perf_counter()
            roll(actions[W: W + K], K)
            t_launch[0] = time.perf_counter() - t0

        elapsed, kernel_s, wall_local = timed(go_head)
        n_err = int(err_count.item())  # the headline rollout's env errors (warmup + timed)
        resets = count_resets(K)
        launch_bytes = rollout_bytes(resets)
        achieved = launch_bytes / kernel_s / 1e9
        head = {
            "elapsed": elapsed, "kernel_s": kernel_s, "wall_local": wall_local, "frac": achieved / HBM_PEAK_GBS,
            "roofline": {
                "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "kernel": ("acx::pack_actions_kernel + " if plan(min(K, T_buf)).packs else "")
                + f"acx::rollout_kernel<{nw_for(L)},{L if L in (36, 128) else 0},4,1>",
                "bytes_per_env_step": step_bytes, "launch_bytes": launch_bytes, "resets_in_launch": resets,
                "launches": n_launch, "kernel_ms": kernel_s * 1e3, "host_launch_ms": t_launch[0] * 1e3,
            },
            "workload": (f"PPO rollout collection (BASELINE configs[2]): {B} envs/GPU, L={L}, horizon {H}, "
                         "cyclical=True, same-step autoreset, full (K,B,2L) int32 obs trajectory; "
                         f"acx_rollout launches of <= {T_buf} steps ({n_launch} for K={K})"),
            "env_errors": n_err,
        }
        del plans

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
        wall, s_d, _ = timed(lambda: go(actions[W: W + K], K))
        nres = count_resets(K)
        nb = rollout_bytes(nres)
        return {"value": seen * B * K / wall, "unit": "env-steps/s", "kernel_ms": s_d * 1e3,
                "ms_per_step": wall / K * 1e3, "resets_per_step": None if nres is None else nres / K,
                "env_errors": int(err_count.item()), "workload": what,
                "roofline": {"bound": "hbm", "achieved": nb / s_d / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": nb / s_d / 1e9 / HBM_PEAK_GBS, "launch_bytes": nb}}

    if do_obs8:
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
        wall8, s8, _ = timed(lambda: go8(actions[W: W + K], K))
        nres = count_resets(K)
        nb8 = rollout_bytes(nres) - K * B * 6 * L  # obs 2L instead of 8L bytes per env-step
        variants["rollout_obs_int8"] = {
            "value": seen * B * K / wall8, "unit": "env-steps/s", "kernel_ms": s8 * 1e3, "ms_per_step": wall8 / K * 1e3,
            "env_errors": int(err_count.item()),
            "workload": "the headline rollout writing the (K,B,2L) observation trajectory as int8 (the reference's "
                        "observation_space dtype) instead of int32",
            "roofline": {"bound": "hbm", "achieved": nb8 / s8 / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": nb8 / s8 / 1e9 / HBM_PEAK_GBS, "launch_bytes": nb8,
                         "bytes_per_env_step": step_bytes - 6 * L}}
        del obs8, st8, cnt8

    if do_desync:
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

    if not rollout_head and not args.no_obs8:
        # config 5's random-action stepping through the fused rollout instead of one call per
        # step: every step's observation is still materialised, as the (K, B, 2L) int8
        # trajectory of VecACEnv.rollout (the reference's observation dtype, ac_env.py:64-70,
        # and what SyncVectorEnv returns), in launches of <= T8 steps reusing the buffers
        T8 = max(1, min(K, 50, (64 << 30) // max(1, B * (2 * L + 6))))
        obs8 = torch.zeros((T8, B, 2 * L), dtype=torch.int8, device=dev)
        rew8 = torch.zeros((T8, B), dtype=torch.int32, device=dev)
        dn8 = torch.zeros((T8, B), dtype=torch.uint8, device=dev)
        tr8 = torch.zeros((T8, B), dtype=torch.uint8, device=dev)
        st8, cnt8 = starts.clone(), torch.zeros(B, dtype=torch.int32, device=dev)
        err_count.zero_()
        n_res8 = [0]

        def go8(a, T, count=False):
            for t0 in range(0, T, T8):
                t1 = min(T, t0 + T8)
                ops.rollout(st8, a[t0:t1], starts, cnt8, horizon=H, cyclical=True, obs_traj=obs8[: t1 - t0],
                            reward_traj=rew8[: t1 - t0], done_traj=dn8[: t1 - t0], trunc_traj=tr8[: t1 - t0],
                            err=err, err_count=err_count)
                if count:
                    n_res8[0] += int((dn8[: t1 - t0] | tr8[: t1 - t0]).sum().item())

        if W > 0:
            go8(actions[:W], W)
        snap8 = (st8.clone(), cnt8.clone())
        go8(actions[W: W + K], K, count=True)  # off the clock: the resets of the timed steps (bytes)
        st8.copy_(snap8[0]), cnt8.copy_(snap8[1])
        del snap8
        err_count.zero_()
        wall8, s8, _ = timed(lambda: go8(actions[W: W + K], K))
        n8 = -(-K // T8)
        # per env-step: action 4 + obs 2L + reward 4 + done 1 + truncated 1; per env per launch
        # state in/out 16L + count in/out 8 + err 1; the starting row (8L) of every reset
        nb8 = K * B * (2 * L + 10) + n8 * B * (16 * L + 9) + n_res8[0] * 8 * L
        variants["stepping_rollout_obs_int8"] = {
            "value": seen * B * K / wall8, "unit": "env-steps/s", "kernel_ms": s8 * 1e3, "ms_per_step": wall8 / K * 1e3,
            "env_errors": int(err_count.item()), "launches": n8,
            "workload": (f"the same random-action walk ({B} envs/GPU, L={L}, horizon {H}, autoreset) through the "
                         f"fused rollout (VecACEnv.rollout), every step's observation written to an int8 (K,B,2L) "
                         f"trajectory, launches of <= {T8} steps"),
            "roofline": {"bound": "hbm", "achieved": nb8 / s8 / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": nb8 / s8 / 1e9 / HBM_PEAK_GBS, "launch_bytes": nb8,
                         "kernel": f"acx::rollout_kernel<{nw_for(L)},{L if L in (36, 128) else 0},4,2>"}}
        del obs8, rew8, dn8, tr8, st8, cnt8

    if not args.no_step_api or not rollout_head:
        # per-call acx_step API: one launch per env step, state in place in HBM, autoreset
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

        def go_steps():
            for t in range(K):
                step(actions[W + t])

        # The in-place step writes back only the relators that changed (gated moves, no-op cyclic
        # conjugations and failed envs leave their rows as they are in HBM), so its bytes depend on
        # the walk: counted over exactly the K timed steps, run first off the clock from a snapshot
        # (the kernel is deterministic, so the timed pass -- and the hipGraph replay below, started
        # from the same snapshot -- takes this same walk).
        snap1 = (st1.clone(), cnt1.clone(), err_count.clone())
        chg = replay_walk(lambda t: step(actions[W + t]), st1, (st1, cnt1, err_count), K, L)["changed"]
        wall_api, s_api, wall_api_local = timed(go_steps)
        n_err_api = int(err_count.item())
        # per env-step: state in 8L + action 4 + count in 4 + changed relators x 4L + lengths 8 +
        # reward 4 + done 1 + truncated 1 + count out 4 + err 1 (SURVEY 8d counts full-row
        # writes, 8L out; the in-place kernel skips unchanged relators, PMC-checked r02h)
        sb = 8 * L + 27 + 4 * L * chg
        step_kernel = ops.step_kernel_name(B, L)
        variants["step_api"] = {
            "value": seen * B * K / wall_api, "unit": "env-steps/s", "ms_per_step": wall_api / K * 1e3,
            "kernel_ms": s_api * 1e3,
            "roofline": {"bound": "hbm", "achieved": B * sb / (s_api / K) / 1e9, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": B * sb / (s_api / K) / 1e9 / HBM_PEAK_GBS, "kernel": step_kernel,
                         "bytes_per_env_step": sb, "changed_relators_per_env_step": chg,
                         "bytes_note": "state read 8L + changed relators x 4L written + 27 B of scalars "
                                       "(in place: unchanged relators are not written); changed relators "
                                       "counted over exactly the timed steps (an untimed replay from a snapshot)"},
            "env_errors": n_err_api,
        }
        # the same walk through the lengths-carrying step (acx_step_lengths), where VecACEnv.step
        # takes it (ops.LENGTHS_STEP_L) or with --workload step; at L = 36 it ties with acx_step
        # (DESIGN.md "The lengths-carrying step") and the default line leaves it out
        run_len = not rollout_head or ops.lengths_step_for(B, L)
        same = True
        if run_len:
            st2 = starts.clone()
            cnt2 = torch.zeros(B, dtype=torch.int32, device=dev)
            lens2 = torch.full((B, 2), L, dtype=torch.int32, device=dev)  # (L, L): read whole, once
            # the rows' reduced flags (acx_step_lengths_reduced, VecACEnv.step's kernel): a
            # conjugation of a row the previous step left reduced reads only its target relator
            red2 = torch.zeros(B, dtype=torch.uint8, device=dev)

            def step2(a):
                ops.step(st2, a, state_out=st2, reset_state=starts, step_count=cnt2, horizon=H, cyclical=True,
                         reward=rew1, done=dn1, truncated=tr1, lengths=lens2, err=err, err_count=err_count,
                         lengths_in=True, reduced=red2)

            def unread(t):
                # the kernel's skip rule (step_body): flag for this mode, a conjugation (ids 4..11),
                # the untouched relator r_{id & 1} of >= 2 letters, no truncation on this step
                a = actions[W + t]
                h = (a & 1).to(torch.int64)
                n_sk = lens2.gather(1, h[:, None])[:, 0]
                ok = (((red2 >> 1) & 1) != 0) & (a >= 4) & (a < 12) & (n_sk >= 2) & (n_sk <= L) & (cnt2 + 1 < H)
                return torch.nn.functional.one_hot(h, 2).bool() & ok[:, None]

            err_count.zero_()
            for t in range(W):
                step2(actions[t])

            def go_steps2():
                for t in range(K):
                    step2(actions[W + t])

            # algorithmic bytes of exactly the timed steps (replayed off the clock from a snapshot):
            # per relator its live 16-byte chunks read (ceil(n/4)), for a changed relator the chunks
            # inside its old or new letters written; + lengths in/out 16 + 27 B of scalars.  The
            # live bytes follow the walk's lengths, which grow through a horizon and drop at the
            # synchronised resets, so a sample of other steps would not do.
            rp = replay_walk(lambda t: step2(actions[W + t]), st2, (st2, cnt2, lens2, red2, err_count), K, L,
                             lens=lens2, unread=unread,
                             finished=(dn1, tr1))
            rd, wr = rp["live_read"], rp["live_written"]
            sb_len = rd + wr + 16 + 27 + 2  # + the reduced flag in and out
            wall_len, s_len, wall_len_local = timed(go_steps2)
            n_err_len = int(err_count.item())
            same = bool(torch.equal(st1, st2))  # both walks took the same W + K steps
            len_kernel = f"acx::step_lengths_kernel<{nw_for(L)},{L if L in (36, 128) else 0},4>"
            a_len = B * sb_len / (s_len / K) / 1e9
            variants["step_api_lengths"] = {
                "value": seen * B * K / wall_len, "unit": "env-steps/s", "ms_per_step": wall_len / K * 1e3,
                "kernel_ms": s_len * 1e3, "env_errors": n_err_len, "same_states_as_step_api": same,
                "roofline": {"bound": "hbm", "achieved": a_len, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": a_len / HBM_PEAK_GBS, "kernel": len_kernel, "bytes_per_env_step": sb_len,
                             "live_bytes_read_per_env_step": rd, "live_bytes_written_per_env_step": wr,
                             "sector_bytes_per_env_step": rp["sector_read"] + rp["sector_written"] + 16 + 29,
                             # the same walk at the memory's read granularity: live chunks read in whole
                             # 128-B lines, plus the starting row each reset env loads whole
                             "line_bytes_per_env_step": rp["line_read"] + wr + 16 + 29 + rp["finished"] * 8 * L,
                             "resets_per_env_step": rp["finished"],
                             "unread_relators_per_env_step": rp["unread"],
                             "bytes_note": "live chunks only: ceil(n/4) x 16 B read per relator the step reads (a "
                                           "conjugation of a row known reduced leaves the other relator unread), "
                                           "changed relators' chunks inside old or new letters written, lengths 16 B "
                                           "+ 27 B of scalars + the reduced flag in and out 2 B, "
                                           "summed over exactly the timed steps (a changed relator's written chunks "
                                           "rounded up to whole 64-B sectors at L = 128, as the kernel writes them); "
                                           "HBM reads whole 128-B lines, so a relator's last live chunk brings its "
                                           "line's dead ones (line_bytes: the same walk at that granularity, plus "
                                           "the starting rows of resets; tools/line_probe.py calibrates it, "
                                           "profiles/r06/r06i_line_probe.json; sector_bytes: 64-B sectors)"},
                "workload": "per-call acx_step_lengths_reduced (VecACEnv.step's path), same walk as step_api",
            }
            if not same:  # a lengths-path regression must not publish a headline
                variants["step_api_lengths"]["error"] = "states differ from acx_step's on the same walk"
            del st2, cnt2, lens2
        if not rollout_head and (not ops.lengths_step_for(B, L) or not same):
            # whole-row tiles (or a lengths walk that left acx_step's states): the headline is acx_step
            a_api = B * sb / (s_api / K) / 1e9
            head = {
                "elapsed": wall_api, "kernel_s": s_api, "wall_local": wall_api_local, "frac": a_api / HBM_PEAK_GBS,
                "roofline": dict(variants["step_api"]["roofline"], kernel_ms=s_api * 1e3, launches=K,
                                 launch_bytes=B * sb),
                "workload": (f"random-action stepping (BASELINE configs[4]): per-call acx_step, {B} envs/GPU, L={L}, "
                             f"horizon {H}, cyclical=True, in-place state, same-step autoreset; {K} launches"),
                "env_errors": n_err_api + (0 if same else 1),
            }
        elif not rollout_head:
            head = {
                "elapsed": wall_len, "kernel_s": s_len, "wall_local": wall_len_local, "frac": a_len / HBM_PEAK_GBS,
                "roofline": dict(variants["step_api_lengths"]["roofline"], kernel_ms=s_len * 1e3, launches=K,
                                 launch_bytes=B * sb_len),
                "workload": (f"random-action stepping (BASELINE configs[4]): per-call acx_step_lengths_reduced (the "
                             f"env's step, ACMove's lengths in/out, per-row reduced flags), {B} envs/GPU, L={L}, horizon {H}, cyclical=True, "
                             f"in-place state, same-step autoreset; {K} launches"),
                "env_errors": n_err_len,
            }

        # the same K per-call steps captured once into a hipGraph (torch.cuda.CUDAGraph over
        # the ctypes launches on the capture stream) and replayed from the timed walk's snapshot:
        # no per-launch host cost, the same bytes as step_api
        if not args.no_graph:
            gs = torch.cuda.Stream(device=dev)
            gs.wait_stream(torch.cuda.current_stream(dev))
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.stream(gs):
                with torch.cuda.graph(graph, stream=gs):
                    go_steps()
            torch.cuda.synchronize()
            restore(snap1, (st1, cnt1, err_count))
            graph.replay()  # warm
            restore(snap1, (st1, cnt1, err_count))
            wall_g, s_g, _ = timed(graph.replay)
            variants["step_api_hipgraph"] = {
                "value": seen * B * K / wall_g, "unit": "env-steps/s", "ms_per_step": wall_g / K * 1e3,
                "kernel_ms": s_g * 1e3, "env_errors": int(err_count.item()),
                "roofline": {"bound": "hbm", "achieved": B * sb / (s_g / K) / 1e9, "peak": HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": B * sb / (s_g / K) / 1e9 / HBM_PEAK_GBS,
                             "bytes_per_env_step": sb},
            }
            del graph
        del snap1

    if not args.no_learner and world == 1:
        # PPO plumbing (acx.agents.LearnerEnv): per step one acx_learner_step launch (int64 policy
        # actions in, float32 obs straight into the learner's (T+1,B,2L) buffer, float32
        # reward/done, episode move history, the round-1 curriculum assignment fused in)
        from acx.agents import LearnerEnv
        KL = min(K, 50)
        lenv = LearnerEnv(np.concatenate([ms_starts(L, B), ms_starts(L, 4096, offset=B)]), B, horizon_length=H,
                          device=dev)
        lobs = torch.empty((KL + 1, B, 2 * L), dtype=torch.float32, device=dev)
        lrew = torch.empty((KL, B), dtype=torch.float32, device=dev)
        ldone = torch.empty((KL, B), dtype=torch.float32, device=dev)
        la = actions[W: W + KL].to(torch.int64)
        lobs.zero_()
        lenv.step(la[0], obs_out=lobs[1], reward_out=lrew[0], done_out=ldone[0])

        def lstep(t):
            lenv.step(la[t], obs_out=lobs[t + 1], reward_out=lrew[t], done_out=ldone[t])

        def go_learn():
            for t in range(KL):
                lstep(t)

        # the learner's own walk, replayed off the clock from a snapshot of every buffer it owns:
        # changed relators and finished envs per env-step of exactly the timed steps
        lbufs = learner_buffers(lenv)
        rp = replay_walk(lstep, lenv.state, lbufs, KL, L, finished=(lenv.done, lenv.truncated))
        _, s_l, _ = timed(go_learn)
        lb = learner_bytes(L, rp["changed"], rp["finished"])
        variants["learner_step"] = {
            "value": B * KL / s_l, "unit": "env-steps/s", "steps": KL, "ms_per_step": s_l / KL * 1e3,
            "roofline": {"bound": "hbm", "achieved": B * lb / (s_l / KL) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": B * lb / (s_l / KL) / 1e9 / HBM_PEAK_GBS, "bytes_per_env_step": lb,
                         "changed_relators_per_env_step": rp["changed"], "finished_per_env_step": rp["finished"],
                         "kernel": f"acx::step_kernel<{nw_for(L)},{L if L in (36, 128) else 0},4,true> "
                                   "(curriculum fused, one launch)",
                         "bytes_note": "16L state read + obs f32 write + 36 B of per-env scalars (move-history "
                                       "ring base included) + changed relators x 4L + per finished env 8L + 8L + "
                                       "8 (curriculum row in, reset row out, curr_index, next ring base) + "
                                       "needs_host 1; counted over exactly the timed steps"},
        }
        # the same with the episodes out of phase (step_count[i] = i mod H, as rollout_desync):
        # ~B/H envs finish and take their next initial state on every step -- a PPO rollout's
        # steady state, where the fused curriculum's ranking is on the path of the tiles that
        # hold finished envs
        del lenv, lbufs
        # an initial-state table long enough that round 1 lasts through the replay and the timed steps
        n_tab = B + 2 * (KL + 1) * (-(-B // H)) + 4096
        lenv = LearnerEnv(ms_starts(L, n_tab), B, horizon_length=H, device=dev)
        lenv.vec.step_count.copy_(torch.arange(B, dtype=torch.int32, device=dev) % H)
        # each env's episode began step_count steps ago: its move-history ring base says so
        lenv.hist_base.copy_((-lenv.vec.step_count) % lenv.hist_cap)
        lenv.step(la[0], obs_out=lobs[1], reward_out=lrew[0], done_out=ldone[0])
        lbufs = learner_buffers(lenv)
        rp2 = replay_walk(lstep, lenv.state, lbufs, KL, L, finished=(lenv.done, lenv.truncated))
        _, s_l2, _ = timed(go_learn)
        lb2 = learner_bytes(L, rp2["changed"], rp2["finished"])
        variants["learner_step_desync"] = {
            "value": B * KL / s_l2, "unit": "env-steps/s", "steps": KL, "ms_per_step": s_l2 / KL * 1e3,
            "roofline": {"bound": "hbm", "achieved": B * lb2 / (s_l2 / KL) / 1e9, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": B * lb2 / (s_l2 / KL) / 1e9 / HBM_PEAK_GBS, "bytes_per_env_step": lb2,
                         "changed_relators_per_env_step": rp2["changed"], "finished_per_env_step": rp2["finished"]},
            "workload": "learner_step with step_count[i] = i mod H: ~B/H finished envs per step take the next "
                        "initial states (round-1 curriculum) inside the step launch"}
        del lobs, lrew, ldone, lenv, lbufs

    if not args.no_config2 and world == 1 and rollout_head:
        variants["config2_step"] = config2_variant(dev, H, timed)

    if not args.no_search and world == 1:
        variants.update(search_variants(dev))

    # HBM traffic per launch from rocprofv3 PMC (FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md
    # "HBM"), measured by profile_cmd.sh on this same command and committed under profiles/;
    # used only when that profile's workload matches this run's.  A profile of the same (B, L, K)
    # gives the launch's measured bytes directly; one of another K is carried over as its
    # measured/algorithmic ratio (the launch's bytes are the same per-step and per-launch terms
    # at any K, so the ratio is K-independent) and labelled as scaled.
    if rollout_head:
        traffic, traffic_src = committed_traffic(B, L, K, head["roofline"]["launch_bytes"])
    else:
        traffic, traffic_src = committed_step_traffic(B, L, head["roofline"]["launch_bytes"],
                                                      head["roofline"].get("kernel", ""))
    head["roofline"].update(traffic=traffic, traffic_source=traffic_src)

    rows = gather_rows([B * K / head["wall_local"], head["kernel_s"] * 1e3, head["frac"], head["wall_local"] * 1e3],
                       dev)
    elapsed = head["elapsed"]
    line = {
        "metric": METRIC,
        "value": seen * B * K / elapsed,
        "unit": "env-steps/s",
        "n_gpus": seen,
        "steps": K,
        "warmup": W,
        "ms_per_step": elapsed / K * 1e3,
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic: Miller-Schupp starting states (all_presentations.txt, env i -> i mod 1190), "
                "uniform random move ids (torch.Generator seed 0+rank)",
        "config": {
            "workload": head["workload"],
            "global_batch": seen * B,
            "envs_per_gpu": B,
            "max_relator_length": L,
            "horizon": H,
            "parallelism": f"env-index shards x{seen}, no data-path collective",
        },
        "world_size_seen": seen,
        "dist_backend": backend if seen > 1 else None,
        "per_rank": _per_rank_rows(rows),
        "roofline": head["roofline"],
        "cpu_baseline": cpus.get("cpu_baseline"),
        "cpu_baseline_c_oracle": cpus.get("cpu_baseline_c_oracle"),
        "cpu_baseline_c_oracle_all_cores": cpus.get("cpu_baseline_c_oracle_all_cores"),
        "variants": variants,
        "env_errors": head["env_errors"],
    }
    if not args.no_bfs:
        run_sharded_bfs_variant(args, line, variants, dev, rank, world, backend)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def profile_tags(suffix: str) -> list:
    """tags of the committed profiles/rNN/<tag>_summary.json whose tag ends in _<suffix>, newest
    first (a round's runs are lettered a..z, then aa..: r06ad > r06u > r06g > r05zz > r05z > r05)"""
    import glob
    tags = [os.path.basename(p)[: -len("_summary.json")]
            for p in glob.glob(os.path.join(REPO, "profiles", "r[0-9][0-9]", f"*_{suffix}_summary.json"))]
    def age(tag):  # r06ad after r06z after r06u after r06 (the letters count up: a..z, then aa..)
        run = tag.split("_")[0]
        letters = run[3:]
        return (run[:3], len(letters), letters)

    return sorted(tags, key=age, reverse=True)


def committed_traffic(B, L, K, launch_bytes):
    """(HBM bytes of the headline launch from the newest committed rocprofv3 PMC profile of this
    workload, where from) or (None, None)"""
    cands = []
    for tag in profile_tags("k20") + ["r04", "r03v", "r03m", "r02o", "r02h", "r02", "r01"]:
        prof = os.path.join(REPO, "profiles", tag.split("_")[0][:3], f"{tag}_summary.json")
        if not os.path.exists(prof):
            continue
        with open(prof) as f:
            ps = json.load(f)
        pc = ps.get("bench_line", {}).get("config", {})
        td = ps.get("rollout_timed_dispatch") or {}
        if pc.get("envs_per_gpu") == B and pc.get("max_relator_length") == L and td.get("pmc_hbm_bytes"):
            cands.append((ps["bench_line"].get("steps") != K, tag, ps["bench_line"].get("steps"), td))
    if not cands:
        return None, None
    scaled, tag, kp, td = min(cands, key=lambda c: c[0])
    where = f"profiles/{tag.split('_')[0][:3]}/{tag}_summary.json: rocprofv3 --pmc FETCH_SIZE (x2) + --pmc WRITE_SIZE"
    if not scaled:
        return td["pmc_hbm_bytes"], f"{where} of this command (K={K})"
    ratio = td["pmc_hbm_bytes"] / td["algorithmic_bytes"]
    return (launch_bytes * ratio,
            f"{where} at K={kp}: measured/algorithmic = {ratio:.4f}, applied to this launch's algorithmic bytes")


def committed_step_traffic(B, L, launch_bytes, kernel):
    """(HBM bytes per step launch, where from) for --workload step: the newest committed
    rocprofv3 PMC profile of the step workload at this (B, L) and of this kernel, as its
    measured/algorithmic ratio applied to this launch's algorithmic bytes (the changed-relator
    rate, hence the bytes, vary slightly with the walk); or (None, None)"""
    want = kernel.replace(" ", "")
    for tag in profile_tags("step128") + profile_tags("step36"):
        prof = os.path.join(REPO, "profiles", tag[:3], f"{tag}_summary.json")
        if not os.path.exists(prof):
            continue
        with open(prof) as f:
            ps = json.load(f)
        pc = ps.get("bench_line", {}).get("config", {})
        rec = ps.get("step_timed_dispatches") or {}
        got = rec.get("kernel", "").split("(")[0].replace("void ", "", 1).replace(" ", "")
        if (pc.get("envs_per_gpu") == B and pc.get("max_relator_length") == L and rec.get("pmc_over_algorithmic")
                and got == want):
            r = rec["pmc_over_algorithmic"]
            return (launch_bytes * r, f"profiles/{tag[:3]}/{tag}_summary.json: rocprofv3 --pmc FETCH_SIZE (x2) + --pmc "
                                      f"WRITE_SIZE per step launch, measured/algorithmic = {r:.4f}")
    return None, None


def config2_variant(dev, H: int, timed) -> dict:
    """BASELINE configs[1]: 65,536 envs, L = 36, Miller-Schupp starts, uniform random move ids
    (device generator, seed 0), per-call step API in place with same-step autoreset (SURVEY 8(d)
    config 2), 200 timed steps after 10 warm-up steps; eager launches and the same 200 launches
    replayed from one hipGraph.  A launch moves ~24 MB: the small-batch step instance
    (ops.step_kernel_name) keeps the whole tile's loads in flight so that the one wave per SIMD
    this batch gives is not exposed three round trips deep."""
    import torch

    from acx import ops

    B2, L2, K2, W2 = 65536, 36, 200, 10
    starts = torch.as_tensor(ms_starts(L2, B2)).to(dev)
    st = starts.clone()
    cnt = torch.zeros(B2, dtype=torch.int32, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    acts = torch.randint(0, 12, (W2 + K2 + 8, B2), dtype=torch.int32, device=dev, generator=g)
    rew = torch.empty(B2, dtype=torch.int32, device=dev)
    dn = torch.empty(B2, dtype=torch.uint8, device=dev)
    tr = torch.empty(B2, dtype=torch.uint8, device=dev)
    lens = torch.empty((B2, 2), dtype=torch.int32, device=dev)
    err = torch.zeros(B2, dtype=torch.uint8, device=dev)
    ec = torch.zeros(1, dtype=torch.int32, device=dev)

    # the arguments resolved once (ops.StepPlan: one ctypes call per step; ops.step's per-call
    # checks, not the ~10 us kernel, set the eager rate at this batch)
    step = ops.StepPlan(st, state_out=st, reset_state=starts, step_count=cnt, horizon=H, cyclical=True, reward=rew,
                        done=dn, truncated=tr, lengths=lens, err=err, err_count=ec)

    for t in range(W2):
        step(acts[t])
    snap = (st.clone(), cnt.clone(), ec.clone())

    # the caller's per-step action tensors exist before the loop (a policy hands each step its
    # own): taking the views here keeps the harness's tensor indexing (~2-3 us of host time per
    # step, more than half the call) out of the timed loop, which then measures StepPlan's call
    views = [acts[W2 + t] for t in range(K2)]

    def go():
        for a_t in views:
            step(a_t)

    # changed relators per env-step (the in-place write-back) over exactly the timed steps, replayed
    # off the clock from the snapshot (the eager and the hipGraph passes both start from it)
    chg = replay_walk(lambda t: step(acts[W2 + t]), st, (st, cnt, ec), K2, L2)["changed"]
    wall, s_k, _ = timed(go)
    n_err = int(ec.item())
    sb = 8 * L2 + 27 + 4 * L2 * chg
    out = {"value": B2 * K2 / wall, "unit": "env-steps/s", "ms_per_step": wall / K2 * 1e3, "kernel_ms": s_k * 1e3,
           "env_errors": n_err, "envs": B2, "steps": K2,
           "roofline": {"bound": "hbm", "achieved": B2 * sb / (s_k / K2) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": B2 * sb / (s_k / K2) / 1e9 / HBM_PEAK_GBS, "bytes_per_env_step": sb,
                        "changed_relators_per_env_step": chg, "kernel": ops.step_kernel_name(B2, L2)},
           "workload": "BASELINE configs[1]: 65536 envs, L=36, Miller-Schupp starts, uniform random actions, per-call "
                       "acx_step in place (ops.StepPlan), horizon 200, same-step autoreset; 200 launches"}
    gs = torch.cuda.Stream(device=dev)
    gs.wait_stream(torch.cuda.current_stream(dev))
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(gs):
        with torch.cuda.graph(graph, stream=gs):
            go()
    torch.cuda.synchronize()
    restore(snap, (st, cnt, ec))
    graph.replay()  # warm
    restore(snap, (st, cnt, ec))
    wall_g, s_g, _ = timed(graph.replay)
    out["hipgraph"] = {"value": B2 * K2 / wall_g, "ms_per_step": wall_g / K2 * 1e3, "kernel_ms": s_g * 1e3,
                       "env_errors": int(ec.item()),
                       "roofline": {"bound": "hbm", "achieved": B2 * sb / (s_g / K2) / 1e9, "peak": HBM_PEAK_GBS,
                                    "unit": "GB/s", "frac": B2 * sb / (s_g / K2) / 1e9 / HBM_PEAK_GBS}}
    del graph
    # the same 65,536 envs through the fused rollout (one launch of 200 steps, full (200, B, 2L)
    # int32 trajectory): the state stays in registers, so the one wave per SIMD is not exposed to
    # a load -> store round trip per step
    restore(snap, (st, cnt, ec))
    obs2 = torch.zeros((K2, B2, 2 * L2), dtype=torch.int32, device=dev)
    rw2 = torch.zeros((K2, B2), dtype=torch.int32, device=dev)
    dn2 = torch.zeros((K2, B2), dtype=torch.uint8, device=dev)
    tr2 = torch.zeros((K2, B2), dtype=torch.uint8, device=dev)
    ec.zero_()

    def roll():
        ops.rollout(st, acts[W2: W2 + K2], starts, cnt, horizon=H, cyclical=True, obs_traj=obs2, reward_traj=rw2,
                    done_traj=dn2, trunc_traj=tr2, err=err, err_count=ec)

    snap2 = (st.clone(), cnt.clone())
    roll()  # warm (compiles nothing; first-touch of the trajectory pages)
    restore(snap2, (st, cnt))
    wall_r, s_r, _ = timed(roll)
    nres = int((dn2 | tr2).sum().item())
    rb = K2 * B2 * (4 + 8 * L2 + 6) + B2 * (16 * L2 + 9) + nres * 8 * L2
    out["rollout"] = {"value": B2 * K2 / wall_r, "ms_per_step": wall_r / K2 * 1e3, "kernel_ms": s_r * 1e3,
                      "env_errors": int(ec.item()),
                      "roofline": {"bound": "hbm", "achieved": rb / s_r / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                   "frac": rb / s_r / 1e9 / HBM_PEAK_GBS, "launch_bytes": rb,
                                   "kernel": f"acx::rollout_kernel<{nw_for(L2)},{L2},4,1>"},
                      "workload": "the same envs and moves, one acx_rollout launch of 200 steps with the full "
                                  "(200, 65536, 2L) int32 trajectory"}
    del obs2, rw2, dn2, tr2
    return out


def search_variants(dev) -> dict:
    """BASELINE configs[3] on one GPU: bfs from AK(3), L = 36, cyclical = False, to 10^7 nodes.
      device_bfs      -- the whole search on the GPU (csrc/acx_bfs.hip), best of 3 wall times;
      expand12_keys   -- the 12-way expansion kernel alone over the first 10^7 BFS nodes
                         (576 B per parent: row in 8L + 12 packed child keys);
      host_dedup_bfs  -- BASELINE's wording, "dedup on host": GPU expansion + the host engine
                         (csrc/acx_search.cpp) replaying the reference's FIFO / dedup / budget;
                         kernel time, kernel + copies, and the host's share reported apart;
      device_greedy   -- greedy_search from AK(3) to 10^6 nodes, visited set in HBM."""
    import torch

    from acx import _lib, ops
    from acx.envs.utils import convert_relators_to_presentation
    from acx.search import _device_bfs as D
    from acx.search import _engine as E
    from acx.search import bfs

    out = {}
    L, nb = 36, 10 ** 7
    ak3 = convert_relators_to_presentation([1, 1, 1, -2, -2, -2, -2], [1, 2, 1, -2, -1, -2], L)
    work = "bfs from AK(3), L=36, cyclical=False, to 10^7 nodes (BASELINE configs[3])"
    try:
        with contextlib.redirect_stdout(io.StringIO()):
            D.device_bfs(ak3, nb, device=dev, keep_node_keys=True)  # warm: workspace, and the node keys
        keys = D.LAST_STATS["node_keys"][:nb]
        walls = []
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            with contextlib.redirect_stdout(io.StringIO()):
                D.device_bfs(ak3, nb, device=dev)
            torch.cuda.synchronize()
            walls.append(time.perf_counter() - t0)
        st = dict(D.LAST_STATS)
        best = min(walls)
        out["device_bfs"] = {"value": st["nodes"] / best, "unit": "BFS nodes/s", "wall_ms": best * 1e3,
                             "walls_ms": [w * 1e3 for w in walls], "nodes": st["nodes"],
                             "parents_expanded": st["parents"], "chunks": st["chunks"], "workload": work + "; device "
                             "visited set (csrc/acx_bfs.hip)"}
        D.release_workspaces()
        kw = _lib.key_words(L)
        parents = ops.unpack_keys(torch.as_tensor(keys.view(np.int64)).to(dev), L)
        N = parents.shape[0]
        kout = {"keys": torch.empty((N, 12, kw), dtype=torch.int64, device=dev)}
        ops.expand12(parents, cyclical=False, children=False, lengths=False, keys=True, err=False, out=kout)
        times = []
        for _ in range(3):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ops.expand12(parents, cyclical=False, children=False, lengths=False, keys=True, err=False, out=kout)
            e1.record()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1) / 1e3)
        best = min(times)
        bpp = 8 * L + 12 * kw * 8
        out["expand12_keys"] = {"value": 12 * N / best, "unit": "children/s", "parents": N, "kernel_ms": best * 1e3,
                                "roofline": {"bound": "hbm", "achieved": N * bpp / best / 1e9, "peak": HBM_PEAK_GBS,
                                             "unit": "GB/s", "frac": N * bpp / best / 1e9 / HBM_PEAK_GBS,
                                             "bytes_per_parent": bpp},
                                "workload": "acx_expand12 keys-only over the first 10^7 nodes of that BFS"}
        del kout, parents, keys
        torch.cuda.empty_cache()
        with contextlib.redirect_stdout(io.StringIO()):
            t0 = time.perf_counter()
            bfs(ak3, nb, device=dev, engine="host")
            wall = time.perf_counter() - t0
        es = dict(E.LAST_STATS)
        host_s = es["host_next_s"] + es["host_store_s"] + es["host_replay_s"]
        out["host_dedup_bfs"] = {
            "value": es["nodes"] / wall, "unit": "BFS nodes/s", "wall_ms": wall * 1e3, "nodes": es["nodes"],
            "parents_expanded": es["expanded"], "rounds": es["rounds"],
            "kernel_ms": es["kernel_s"] * 1e3,
            "kernel_children_per_s": 12 * es["expanded"] / es["kernel_s"],
            "kernel_d2h_ms": es["gpu_roundtrip_s"] * 1e3,
            "kernel_d2h_children_per_s": 12 * es["expanded"] / es["gpu_roundtrip_s"],
            "host_dedup_ms": host_s * 1e3,
            "end_to_end_children_per_s": 12 * es["expanded"] / wall,
            "workload": work + "; dedup on host (engine='host'): kernel_ms = unpack + expand12 on the GPU, "
                               "kernel_d2h_ms = + H2D parents / D2H child keys per batch, host_dedup_ms = the host "
                               "engine's pop / store / replay"}
        # the other half of configs[3]: greedy_search from AK(3) (greedy.py:15-121) to 10^6 nodes,
        # the visited set in HBM (csrc/acx_greedy.hip), pops replayed on the host in the reference's
        # order; best of 2 wall times after a warm-up
        from acx.search import greedy_search

        ng = 10 ** 6
        with contextlib.redirect_stdout(io.StringIO()):
            greedy_search(ak3, ng, device=dev)
        gw = []
        for _ in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            with contextlib.redirect_stdout(io.StringIO()):
                gres = greedy_search(ak3, ng, device=dev)
            gw.append(time.perf_counter() - t0)
        gs = dict(E.LAST_STATS)
        out["device_greedy"] = {
            "value": gs["nodes"] / min(gw), "unit": "search nodes/s", "wall_ms": min(gw) * 1e3,
            "walls_ms": [w * 1e3 for w in gw], "nodes": gs["nodes"], "pops": gs["pops"], "rounds": gs["rounds"],
            "expanded": gs["expanded"], "gpu_roundtrip_ms": gs["gpu_roundtrip_s"] * 1e3,
            "host_replay_ms": gs["host_replay_s"] * 1e3, "result": [bool(gres[0]), len(gres[1]) if gres[1] else None],
            "workload": "greedy_search from AK(3), L=36, cyclical=False, to 10^6 nodes (BASELINE configs[3], "
                        "greedy half); visited set in HBM (csrc/acx_greedy.hip), host replays the pop order"}
    except Exception as e:  # noqa: BLE001 -- a variant: its failure must not cost the headline line
        out["search_error"] = repr(e)[:300]
    return out


class LineGuard:
    """World > 1, around the sharded-BFS variant: the measured line reaches stdout even if that
    variant never returns.  Two triggers make rank 0 print the line (the variant marked with what
    happened) and end the process with EXIT_BFS_STALL:
      * a deadline of `timeout_s` (a stalled exchange);
      * a signal -- SIGTERM is what torchrun sends the surviving ranks when another rank dies (a
        fault inside its collective, say).  It arrives through signal.set_wakeup_fd, so a helper
        thread sees it while the main thread is blocked inside a C call (an RCCL wait, a ctypes
        call), where a Python-level handler would not run until that call returned.
    Leaving the block normally disarms both.  Main thread only (signal handlers)."""

    def __init__(self, line: dict, variants: dict, key: str, rank: int, timeout_s: float):
        self.line, self.variants, self.key, self.rank, self.timeout_s = line, variants, key, rank, timeout_s

    def __enter__(self):
        import signal
        import threading

        self._r, self._w = os.pipe()
        self._cr, self._cw = os.pipe()  # disarm
        os.set_blocking(self._w, False)
        self._old_fd = signal.set_wakeup_fd(self._w)
        self._old_h = signal.signal(signal.SIGTERM, lambda *_: None)  # no-op: the helper thread acts
        self._t = threading.Thread(target=self._watch, daemon=True)
        self._t.start()
        return self

    def _fire(self, why: str) -> None:
        if self.rank == 0:  # the variant may be inside redirect_stdout: write to the real stdout
            self.variants[self.key] = {"error": why}
            sys.__stdout__.write(json.dumps(self.line) + "\n")
            sys.__stdout__.flush()
        os._exit(EXIT_BFS_STALL)

    def _watch(self) -> None:
        import select
        import signal

        ready, _, _ = select.select([self._r, self._cr], [], [], self.timeout_s)
        if self._cr in ready:
            return
        if self._r in ready:
            sig = os.read(self._r, 1)
            name = signal.Signals(sig[0]).name if sig and sig[0] in signal.Signals._value2member_map_ else "a signal"
            self._fire(f"aborted by {name} (torchrun stops the surviving ranks when one exits)")
        self._fire(f"timeout after {self.timeout_s:.0f} s")

    def __exit__(self, *exc):
        import signal

        os.write(self._cw, b"x")
        self._t.join()
        signal.signal(signal.SIGTERM, self._old_h)
        signal.set_wakeup_fd(self._old_fd)
        for fd in (self._r, self._w, self._cr, self._cw):
            os.close(fd)
        return False


def run_sharded_bfs_variant(args, line, variants, dev, rank, world, backend) -> None:
    """BASELINE configs[3] on the owner-partitioned BFS (csrc/acx_sbfs.hip): AK(3), L = 36, to 10^7
    nodes; node store + visited set sharded over the ranks by key owner, per-chunk RCCL
    all_gather / all_to_all / all_reduce (world 1: the exchanges are local copies).  Last, behind
    a guard: the one variant with collectives on its data path.  At world > 1 (LineGuard) a stalled
    exchange, or the SIGTERM torchrun sends when another rank dies, makes rank 0 print the line with
    the variant marked and every rank exit with EXIT_BFS_STALL: a failure there costs neither the
    headline line nor a visible failure status."""
    import torch

    from acx.envs.utils import convert_relators_to_presentation
    from acx.search import _sharded_bfs as SB

    guard = LineGuard(line, variants, "sharded_bfs", rank, args.bfs_timeout) if world > 1 else contextlib.nullcontext()
    with guard:
        try:
            ak3 = convert_relators_to_presentation([1, 1, 1, -2, -2, -2, -2], [1, 2, 1, -2, -1, -2], 36)
            nb = 10 ** 7
            with contextlib.redirect_stdout(io.StringIO()):
                SB.sharded_bfs(ak3, nb, device=dev)  # warmup: workspace allocation
            if os.environ.get("ACX_BENCH_KILL_RANK") == str(rank):  # rehearsal hook (tools/gpu_n2_rehearsal.sh)
                os._exit(7)  # a rank dying mid-variant: the others must still produce the line
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
            variants["sharded_bfs"] = {
                "value": st["nodes"] / best, "unit": "BFS nodes/s", "wall_ms": best * 1e3, "nodes": st["nodes"],
                "parents_expanded": st["parents"], "chunks": st["chunks"], "result": list(res) if res[0] else [False, None],
                "workload": "BASELINE configs[3]: bfs from AK(3), L=36, cyclical=False, to 10^7 nodes; node store and "
                            f"visited set partitioned by key owner over {world} rank(s), "
                            f"{'RCCL' if backend == 'nccl' else backend} exchanges per chunk",
            }
        except Exception as e:  # noqa: BLE001 -- a variant (failing the same on every rank)
            variants["sharded_bfs"] = {"error": repr(e)[:300]}
    SB.release_workspaces()


if __name__ == "__main__":
    main()
