"""Store-stream probe (tools/store_throttle.hip) on ONE (K, B, 2L) int32 trajectory buffer
(K = 20, B = 2^20, L = 36: 6.04 GB), every pattern interleaved REPS times with the bench's own
K = 20 rollout writing the same buffer, HIP events on the current stream.  Hypothesis: the
rollout's store rate (5.1-5.3 TB/s on slow boxes, vs ~7 for a one-shot fill of the same rows) is
set by how many stores each long-lived wave keeps in flight; if a throttled tile pattern writes
at the fill's rate, the rollout's obs store gets the same throttle.

    python tools/store_throttle.py [--reps 5] [--spin 0,200]
"""
import argparse
import ctypes
import json
import os
import statistics
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "ac-solver-caltech_amd"))
from bench import ms_starts  # noqa: E402


def lib():
    so = os.path.join(HERE, "libstore_throttle.so")
    src = os.path.join(HERE, "store_throttle.hip")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.check_call(["hipcc", "-O3", "--offload-arch=gfx950", "-shared", "-fPIC", src, "-o", so])
    L = ctypes.CDLL(so)
    L.probe_store.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                              ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--spin", default="0,200")
    ap.add_argument("--throttle", default="0,1,2,4,8,16", type=lambda x: [int(v) for v in x.split(",")])
    ap.add_argument("--K", type=int, default=20, help="steps per launch (trajectory rows K x B)")
    ap.add_argument("--only", default="", help="comma-separated case names to run (default: all)")
    a = ap.parse_args()
    K, B, L, H = a.K, 1 << 20, 36, 200
    dev = torch.device("cuda:0")
    P = lib()
    import acx  # noqa: F401
    from acx import ops

    obs = torch.zeros((K, B, 2 * L), dtype=torch.int32, device=dev)
    starts = torch.as_tensor(ms_starts(L, B)).to(dev)
    state = torch.empty_like(starts)
    cnt = torch.zeros(B, dtype=torch.int32, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    acts = torch.randint(0, 12, (K, B), dtype=torch.int32, device=dev, generator=g)
    rew = torch.zeros((K, B), dtype=torch.int32, device=dev)
    dn = torch.zeros((K, B), dtype=torch.uint8, device=dev)
    tr = torch.zeros((K, B), dtype=torch.uint8, device=dev)
    plan = ops.RolloutPlan(state, starts, cnt, T=K, horizon=H, cyclical=True, obs_traj=obs, reward_traj=rew,
                           done_traj=dn, trunc_traj=tr)
    props = torch.cuda.get_device_properties(dev)
    resident = props.multi_processor_count * 8  # 8 blocks of 4 waves per CU = 8 waves per SIMD
    nbytes = obs.numel() * 4
    spins = [int(x) for x in a.spin.split(",")]
    cases = [(f"rollout_k{K}", None)]
    cases += [("fill_oneshot", (0, 0, 0)), ("tile_oneshot", (3, 0, 0))]
    cases += [(f"fill_stride_n{n}", (1, n, 0)) for n in a.throttle]
    cases += [(f"tile_n{n}_spin{s}", (2, n, s)) for s in spins for n in a.throttle]
    cases += [(f"tile_grouped{ge}", (4, ge, 0)) for ge in (8, 16, 32)]
    cases += [(f"tile_cpol{pol}", (5, pol, 0)) for pol in (0, 1, 2, 16, 17, 18)]
    cases += [("tile_block", (6, 0, 0)), ("tile_block_sync", (6, 1, 0)), ("tile_block_oneshot", (7, 0, 0))]
    cases += [(f"tile_rot{r}", (8, r, 0)) for r in (1, 5, 7)]
    cases += [("tile_desync", (9, 0, 0))]
    if a.only:
        keep = set(a.only.split(","))
        cases = [(n, c) for n, c in cases if n in keep]
    ms = {c: [] for c, _ in cases}
    for rep in range(a.reps + 1):
        for name, c in cases:
            torch.cuda.synchronize()
            s = torch.cuda.current_stream().cuda_stream
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            if c is None:
                state.copy_(starts)
                cnt.zero_()
                e0.record()
                plan(acts)
            else:
                e0.record()
                rc = P.probe_store(c[0], c[1], obs.data_ptr(), B, L, K, c[2], resident, s)
                assert rc == 0, rc
            e1.record()
            torch.cuda.synchronize()
            if rep:
                ms[name].append(e0.elapsed_time(e1))
    out = {"what": f"tools/store_throttle.py: store patterns on one ({K}, 2^20, 72) int32 buffer, "
                   "interleaved, medians; TB/s = buffer bytes / time (the rollout also moves ~0.9 GB of "
                   "state / ids / rewards, not counted here)",
           "K": K, "resident_blocks": resident, "buffer_bytes": nbytes, "cases": {}}
    for name, v in ms.items():
        m = statistics.median(v)
        out["cases"][name] = {"ms": round(m, 4), "TBps": round(nbytes / m / 1e9, 3), "all_ms": [round(x, 4) for x in v]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
