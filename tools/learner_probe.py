"""Where the steady-state learner step's time goes (bench.py's learner_step_desync workload).

2^20 envs, L = 36, horizon 200, step_count[i] = i mod H (≈ B/H envs finish per step and take
the next initial states of the round-1 curriculum).  From one snapshot of the LearnerEnv's
buffers, K steps are timed (HIP events, current stream) through
  fused  -- acx_learner_step (one launch, the ranking inside the step kernel),
  four   -- acx_step_learner + acx_curriculum_assign,
  fused_nohist -- fused without the per-env move history (hist_cap 0),
and the same two on the fresh workload (every step_count 0: almost no env finishes).  Every
variant must leave the same state (checksum).  Run under rocprofv3 --kernel-trace --stats to
split the four-launch path by kernel.

    python tools/learner_probe.py [--K 50] [--reps 3] [--libs a.so b.so ...]

--libs: the fused step through each library in turn (tools/ab_build.sh builds: kernels and
curriculum only), same buffers, interleaved, as "fused@<name>".
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "ac-solver-caltech_amd"))
from bench import learner_buffers, ms_starts, restore  # noqa: E402


class _Null:
    """a NULL device pointer where LearnerEnv passes action_hist.data_ptr()"""

    def data_ptr(self):
        return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=50)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--B", type=int, default=1 << 20)
    ap.add_argument("--libs", nargs="*", default=[])
    args = ap.parse_args()
    import ctypes

    from acx import _lib
    from acx.agents import LearnerEnv

    main_lib = _lib.load()
    libs = {"": main_lib}
    for path in args.libs:
        lib = ctypes.CDLL(os.path.abspath(path))
        for name, (argtypes, restype) in _lib.SIGNATURES.items():
            if hasattr(lib, name):
                getattr(lib, name).argtypes = argtypes
                getattr(lib, name).restype = restype
        libs[os.path.basename(path)] = lib
    modes = [("fused", ""), ("four", ""), ("fused_nohist", "")] if not args.libs else \
        [("fused", k) for k in libs]

    dev = torch.device("cuda:0")
    L, H, B, K = 36, 200, args.B, args.K
    g = torch.Generator(device=dev).manual_seed(0)
    acts = torch.randint(0, 12, (K, B), generator=g, device=dev, dtype=torch.int64)
    obs = torch.empty((K + 1, B, 2 * L), dtype=torch.float32, device=dev)
    rew = torch.empty((K, B), dtype=torch.float32, device=dev)
    done = torch.empty((K, B), dtype=torch.float32, device=dev)
    res = {"B": B, "L": L, "K": K}
    for wl in ("desync", "fresh"):
        n_tab = B + 2 * (K + 1) * (-(-B // H)) * args.reps * 2 + 4096
        lenv = LearnerEnv(ms_starts(L, n_tab), B, horizon_length=H, device=dev)
        # a workspace large enough for every library's layout (acx_curriculum_workspace may differ)
        lenv._ws = torch.zeros(max(int(lib.acx_curriculum_workspace(B)) for lib in libs.values()), dtype=torch.int32,
                               device=dev)
        if wl == "desync":
            lenv.vec.step_count.copy_(torch.arange(B, dtype=torch.int32, device=dev) % H)
            lenv.hist_base.copy_((-lenv.vec.step_count) % lenv.hist_cap)
        lenv.step(acts[0], obs_out=obs[1], reward_out=rew[0], done_out=done[0])
        hist_cap, hist, hbase = lenv.hist_cap, lenv.action_hist, lenv.hist_base
        bufs = learner_buffers(lenv)
        snap = [t.clone() for t in bufs]
        torch.cuda.synchronize()
        sums = {}
        for rep in range(args.reps):
            for mode, lk in modes:
                _lib._lib = libs[lk]
                # fused_nohist: hist_cap 0 -- the kernel writes no move history (isolates the cost of
                # the (hist_cap, B) byte writes, one cache line per lane when episodes are out of phase)
                lenv.hist_cap = 0 if mode == "fused_nohist" else hist_cap
                lenv.action_hist = _Null() if mode == "fused_nohist" else hist
                lenv.hist_base = _Null() if mode == "fused_nohist" else hbase
                restore(snap, bufs)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for t in range(K):
                    lenv.step(acts[t], obs_out=obs[t + 1], reward_out=rew[t], done_out=done[t], fused=mode != "four")
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / K
                fin = int(lenv.done.sum().item() + lenv.truncated.sum().item())
                ck = int(lenv.state.to(torch.int64).sum().item())
                if sums.setdefault("ref", ck) != ck:  # every mode and rep leaves the same state
                    res[f"{wl}_mismatch"] = True
                _lib._lib = main_lib
                res.setdefault(f"{wl}_{mode}{'@' + lk if lk else ''}_ms", []).append(round(ms, 4))
                res[f"{wl}_finished_last_step"] = fin
        del lenv, bufs, snap
    print(json.dumps(res))


if __name__ == "__main__":
    main()
