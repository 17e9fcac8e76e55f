"""In-process A/B of rollout builds (tools/ab_build.sh): the bench's K = 20 rollout (2^20 envs,
L = 36, Miller-Schupp starts, horizon 200, packed ids, full int32 and int8 obs trajectories) run
through each library in turn on the SAME buffers, REPS rounds interleaved, HIP events on the
current stream.  Same buffers and interleaving take allocation placement out of the comparison.

    python tools/ab_rollout.py abv/libacx_base.so abv/libacx_x.so ... [--reps N] [--obs 32|8|both]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from bench import ms_starts  # noqa: E402

P = ctypes.c_void_p
I32, I64 = ctypes.c_int32, ctypes.c_int64


def load(path):
    lib = ctypes.CDLL(os.path.abspath(path))
    lib.acx_pack_actions.argtypes = [P, P, I32, I64, P]
    lib.acx_rollout_packed.argtypes = [P] * 10 + [I32, I64, I32, I32, I32, P]
    lib.acx_rollout_obs8.argtypes = [P] * 11 + [I32, I64, I32, I32, I32, P]
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--K", default="20", help="steps per launch; a comma list runs each K on the same buffers")
    ap.add_argument("--obs", default="both")
    ap.add_argument("--no-check", action="store_true",
                    help="timing-only variants that skip work on purpose (outputs not compared)")
    a = ap.parse_args()
    # each entry "T" or "T@S": a T-step launch writing trajectory rows [S, S + T) of the buffer
    Ks = [(int(x.split("@")[0]), int(x.split("@")[1]) if "@" in x else 0) for x in a.K.split(",")]
    K, B, L, H = max(t + o for t, o in Ks), 1 << 20, 36, 200
    dev = torch.device("cuda:0")
    libs = [(os.path.basename(p), load(p)) for p in a.libs]
    starts = torch.as_tensor(ms_starts(L, B)).to(dev)
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    acts = torch.randint(0, 12, (K, B), dtype=torch.int32, device=dev, generator=g)
    pk = torch.empty(((K + 7) // 8, B), dtype=torch.int32, device=dev)
    rew = torch.zeros((K, B), dtype=torch.int32, device=dev)
    dn = torch.zeros((K, B), dtype=torch.uint8, device=dev)
    tr = torch.zeros((K, B), dtype=torch.uint8, device=dev)
    err = torch.zeros(B, dtype=torch.uint8, device=dev)
    ec = torch.zeros(1, dtype=torch.int32, device=dev)
    o32 = torch.zeros((K, B, 2 * L), dtype=torch.int32, device=dev)
    o8 = torch.zeros((K, B, 2 * L), dtype=torch.int8, device=dev)
    state = torch.empty_like(starts)
    cnt = torch.zeros(B, dtype=torch.int32, device=dev)
    kinds = ["i32", "i8"] if a.obs == "both" else (["i32"] if a.obs == "32" else ["i8"])
    ms = {(n, k, T, off): [] for n, _ in libs for k in kinds for T, off in Ks}
    ref = {}
    for rep in range(a.reps + 1):
        for n, lib in libs:
            for k in kinds:
              for T, off in Ks:
                  state.copy_(starts)
                  cnt.zero_()
                  ec.zero_()
                  torch.cuda.synchronize()
                  s = torch.cuda.current_stream().cuda_stream
                  e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                  e0.record()
                  assert lib.acx_pack_actions(acts.data_ptr(), pk.data_ptr(), T, B, s) == 0
                  if k == "i32":
                      rc = lib.acx_rollout_packed(state.data_ptr(), pk.data_ptr(), starts.data_ptr(), cnt.data_ptr(),
                                                  o32[off].data_ptr(), rew.data_ptr(), dn.data_ptr(), tr.data_ptr(),
                                                  err.data_ptr(), ec.data_ptr(), T, B, L, H, 1, s)
                  else:
                      rc = lib.acx_rollout_obs8(state.data_ptr(), None, pk.data_ptr(), starts.data_ptr(), cnt.data_ptr(),
                                                o8[off].data_ptr(), rew.data_ptr(), dn.data_ptr(), tr.data_ptr(),
                                                err.data_ptr(), ec.data_ptr(), T, B, L, H, 1, s)
                  e1.record()
                  torch.cuda.synchronize()
                  assert rc == 0 and int(ec.item()) == 0, (n, k, rc, int(ec.item()))
                  if rep > 0:
                      ms[(n, k, T, off)].append(e0.elapsed_time(e1))
                  # every build must produce the same trajectory (checksums of the outputs)
                  o = o32 if k == "i32" else o8
                  sig = (int(o[off:off + T].sum(dtype=torch.int64)), int(rew[:T].sum(dtype=torch.int64)), int(state.sum(dtype=torch.int64)))
                  ref.setdefault((k, T), sig)
                  assert a.no_check or ref[(k, T)] == sig, (n, k, T, sig, ref[(k, T)])
    # the same trajectory rows written by torch's fill_ (a one-pass linear write): their store rate
    out = {}
    for T, off in Ks:
        fills = []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            o32[off:off + T].fill_(1)
            e1.record()
            torch.cuda.synchronize()
            fills.append(e0.elapsed_time(e1))
        f = statistics.median(fills)
        out[f"fill_i32_K{T}@{off}"] = {"median_ms": round(f, 4), "TB_s": round(T * B * 8 * L / (f * 1e-3) / 1e12, 3)}
    state_b = B * (16 * L + 8 + 1)
    for (n, k, T, off), v in ms.items():
        per = 6.5 + (8 * L if k == "i32" else 2 * L)
        nbytes = T * B * per + state_b
        med = statistics.median(v)
        out[f"{n}:{k}:K{T}@{off}"] = {"median_ms": round(med, 4), "min_ms": round(min(v), 4), "all": [round(x, 4) for x in v],
                           "frac_median": round(nbytes / (med * 1e-3) / 1e9 / 8000, 4)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
