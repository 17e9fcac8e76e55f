"""Interleaved A/B of libacx.so builds in ONE process (cdna_hip_programming.md rule 24).

    python tools/ab_libs.py libA.so libB.so [--reps 7] [--mode rollout|step|expand] [--T 200]
                            [--desync] [--unpacked]

Each build gets its own ctypes handle (RTLD_LOCAL); all time the same rollout (B = 2^20,
L = 36, T steps, all outputs; acx_pack_actions + acx_rollout_packed as bench.py does, or
acx_rollout with --unpacked), T acx_step launches, or an expand12 pass, alternating.
--desync starts the step counts at i mod H (scattered resets) instead of 0."""
import argparse
import ctypes
import json
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ac-solver-caltech_amd"))
sys.path.insert(0, REPO)
from bench import ms_starts  # noqa: E402
from acx import _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("libs", nargs="+")
ap.add_argument("--reps", type=int, default=7)
ap.add_argument("--mode", default="rollout")
ap.add_argument("--T", type=int, default=200)
ap.add_argument("--L", type=int, default=36)
ap.add_argument("--rounds", type=int, default=1, help="fresh output allocations (the speed depends on the mapping)")
ap.add_argument("--desync", action="store_true")
ap.add_argument("--unpacked", action="store_true")
args = ap.parse_args()

libs = []
for p in args.libs:
    lib = ctypes.CDLL(os.path.abspath(p))
    for name, (at, rt) in _lib.SIGNATURES.items():
        if hasattr(lib, name):
            getattr(lib, name).argtypes = at
            getattr(lib, name).restype = rt
    libs.append(lib)

dev = torch.device("cuda:0")
L, B, T, H = args.L, 1 << 20, args.T, 200
starts = torch.as_tensor(ms_starts(L, B)).to(dev)
g = torch.Generator(device=dev)
g.manual_seed(0)
acts = torch.randint(0, 12, (T, B), dtype=torch.int32, device=dev, generator=g)
packed = torch.empty(((T + 7) // 8, B), dtype=torch.int32, device=dev)
lens = torch.zeros((B, 2), dtype=torch.int32, device=dev)
stream = torch.cuda.current_stream().cuda_stream


def run(lib):
    state = starts.clone()
    cnt = (torch.arange(B, dtype=torch.int32, device=dev) % H) if args.desync else torch.zeros(B, dtype=torch.int32, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    if args.mode == "rollout" and args.unpacked:
        rc = lib.acx_rollout(state.data_ptr(), acts.data_ptr(), starts.data_ptr(), cnt.data_ptr(), obs.data_ptr(),
                             rew.data_ptr(), dn.data_ptr(), tr.data_ptr(), None, None, T, B, L, H, 1, stream)
        assert rc == 0
    elif args.mode == "rollout":
        rc = lib.acx_pack_actions(acts.data_ptr(), packed.data_ptr(), T, B, stream)
        assert rc == 0
        rc = lib.acx_rollout_packed(state.data_ptr(), packed.data_ptr(), starts.data_ptr(), cnt.data_ptr(),
                                    obs.data_ptr(), rew.data_ptr(), dn.data_ptr(), tr.data_ptr(), None, None, T, B, L,
                                    H, 1, stream)
        assert rc == 0
    elif args.mode == "expand":  # config 4's kernel: 12 packed child keys per parent (search setting)
        rc = lib.acx_expand12(exp_par.data_ptr(), None, None, exp_keys.data_ptr(), None, None, exp_par.shape[0], L, 0,
                              stream)
        assert rc == 0
    else:
        for t in range(T):
            rc = lib.acx_step(state.data_ptr(), state.data_ptr(), acts[t].data_ptr(), starts.data_ptr(),
                              cnt.data_ptr(), rew[t].data_ptr(), dn[t].data_ptr(), tr[t].data_ptr(),
                              lens.data_ptr(), None, None, None, B, L, H, 1, stream)
            assert rc == 0
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


if args.mode == "expand":  # 2^23 parents: random walks off the starting states
    exp_par = starts.repeat(8, 1).contiguous()
    for _k in range(16):
        rc = libs[0].acx_step(exp_par.data_ptr(), exp_par.data_ptr(),
                              torch.randint(0, 12, (exp_par.shape[0],), dtype=torch.int32, device=dev).data_ptr(),
                              None, None, None, None, None, None, None, None, None, exp_par.shape[0], L, H, 0, stream)
        assert rc == 0
    exp_keys = torch.empty((exp_par.shape[0], 12, _lib.key_words(L)), dtype=torch.int64, device=dev)
times = [[] for _ in libs]
for rnd in range(args.rounds):
    obs = torch.zeros((T, B, 2 * L), dtype=torch.int32, device=dev)
    rew = torch.zeros((T, B), dtype=torch.int32, device=dev)
    dn = torch.zeros((T, B), dtype=torch.uint8, device=dev)
    tr = torch.zeros((T, B), dtype=torch.uint8, device=dev)
    for lib in libs:  # warm up each build
        run(lib)
    for r in range(args.reps):
        for i, lib in enumerate(libs):
            times[i].append(run(lib))
    del obs, rew, dn, tr
    torch.cuda.empty_cache()
out = {os.path.basename(p): {"ms_min": min(t), "ms_median": statistics.median(t), "all": [round(x, 2) for x in t]} for p, t in zip(args.libs, times)}
print(json.dumps(out))
