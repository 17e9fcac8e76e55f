"""Where config 2's step time goes (BASELINE configs[1]: 65,536 envs, L = 36).  Every entry is K
back-to-back launches between two HIP events on one stream, driven through ctypes (a few us of
host time per call, below the kernel's), so the per-launch figure is the kernel's duration plus
the gap between launches:
  * the in-place step (acx_step, as bench.py's config2_step) through each library given, at
    several batch sizes -- the fixed part of a launch against the per-env part -- and at 65,536
    with every move id invalid (no move, no write-back);
  * the bare kernels of tools/stream_ceiling.hip at the step's grid: an empty kernel (the launch
    floor), the step's tile reads alone, reads + a quarter written back.

    python tools/config2_probe.py LIB [LIB ...] [--K 200] [--reps 5]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)
from ab_step import ceiling_lib, load  # noqa: E402
from bench import ms_starts  # noqa: E402


def timed(fn, K, reps):
    out = []
    for r in range(reps + 1):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for t in range(K):
            fn(t)
        e1.record()
        torch.cuda.synchronize()
        if r:
            out.append(e0.elapsed_time(e1) / K * 1e3)
    return {"us_per_launch": round(statistics.median(out), 3), "min": round(min(out), 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--K", type=int, default=200)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    L, K, H = 36, a.K, 200
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    res = {"L": L, "K": K}
    for B in (16384, 65536, 131072, 262144, 1 << 20):
        starts = torch.as_tensor(ms_starts(L, B)).to(dev)
        st = starts.clone()
        cnt = torch.zeros(B, dtype=torch.int32, device=dev)
        g = torch.Generator(device=dev)
        g.manual_seed(0)
        acts = torch.randint(0, 12, (K, B), dtype=torch.int32, device=dev, generator=g)
        bad = torch.full((B,), 12, dtype=torch.int32, device=dev)
        rew = torch.empty(B, dtype=torch.int32, device=dev)
        dn = torch.empty(B, dtype=torch.uint8, device=dev)
        tr = torch.empty(B, dtype=torch.uint8, device=dev)
        lens = torch.empty((B, 2), dtype=torch.int32, device=dev)
        err = torch.zeros(B, dtype=torch.uint8, device=dev)
        for path in a.libs:
            lib = load(path)
            name = os.path.basename(path)

            def step(t, ids=None):
                a_ = acts[t] if ids is None else ids
                rc = lib.acx_step(st.data_ptr(), st.data_ptr(), a_.data_ptr(), starts.data_ptr(), cnt.data_ptr(),
                                  rew.data_ptr(), dn.data_ptr(), tr.data_ptr(), lens.data_ptr(), None, err.data_ptr(),
                                  None, B, L, H, 1, s)
                assert rc == 0, rc

            st.copy_(starts)
            cnt.zero_()
            print(f"B{B} {name}", file=sys.stderr, flush=True)
            res[f"B{B}_{name}"] = timed(step, K, a.reps)
            if B == 65536:
                res[f"B{B}_{name}_invalid_ids"] = timed(lambda t: step(t, bad), K, a.reps)
        if B in (65536, 1 << 20):  # the bare shapes at config 2's batch and at the headline's
            cl = ceiling_lib()
            out = torch.zeros(16384, dtype=torch.int32, device=dev)
            for kind, nm in ((5, "empty"), (1, "read_tile"), (3, "rw_tile"), (2, "read_tile_pipe")):
                print(f"B{B} ceiling {nm}", file=sys.stderr, flush=True)
                for lds, occ in ((20 * 1024, 8),):
                    res[f"B{B}_{nm}_nb16"] = timed(
                        lambda t: cl.probe_run(kind, 16, st.data_ptr(), B, L, lds, out.data_ptr(), s), K, a.reps)
        del starts, st, acts
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
