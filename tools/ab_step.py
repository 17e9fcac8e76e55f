"""In-process A/B of in-place step builds (tools/ab_build.sh with L128=1 for L = 128), plus the
streaming ceilings of the same state (tools/stream_ceiling.hip).

The bench's step_api variant: 2^20 envs, Miller-Schupp starts, uniform moves, horizon 200,
in-place state, autoreset; K per-call acx_step launches timed with HIP events on the current
stream, each library in turn on the SAME buffers, REPS rounds interleaved; every library must
leave the same state / counts / rewards (checksums).  Bytes per env-step as bench.py's
step_api (state read 8L + changed relators x 4L + 27 B), with the changed-relator rate measured.

    python tools/ab_step.py abv/libacx_a.so abv/libacx_b.so ... [--L 128] [--K 20] [--reps 5] [--ceiling]

An entry LIB@lengths steps through acx_step_lengths (the rows' lengths carried from call to call,
set from the rows before the warmup), LIB@LL through acx_step_lengths with every row's lengths
reset to (L, L) -- "read the whole row" -- before each call (the refill is a separate timed
launch, reported apart): the cost of the lengths dependency without the byte saving.
LIB@reduced steps through acx_step_lengths_reduced (lengths and per-row reduced flags carried;
a conjugation of a known-reduced row leaves the other relator unread).
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
from bench import ms_starts  # noqa: E402

P = ctypes.c_void_p
I32, I64 = ctypes.c_int32, ctypes.c_int64
PEAK = 8000.0


def load(path):
    lib = ctypes.CDLL(os.path.abspath(path))
    lib.acx_step.argtypes = [P] * 12 + [I64, I32, I32, I32, P]
    if hasattr(lib, "acx_step_lengths"):
        lib.acx_step_lengths.argtypes = [P] * 11 + [I64, I32, I32, I32, P]
    if hasattr(lib, "acx_step_lengths_reduced"):
        lib.acx_step_lengths_reduced.argtypes = [P] * 12 + [I64, I32, I32, I32, P]
    return lib


def ceiling_lib():
    so = os.path.join(HERE, "libstream_ceiling.so")
    if not os.path.exists(so):
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-shared", "-fPIC",
                               os.path.join(HERE, "stream_ceiling.hip"), "-o", so])
    lib = ctypes.CDLL(so)
    lib.probe_run.argtypes = [I32, I32, P, I64, I32, I32, P, P]
    return lib


def ceilings(L, B, reps, dev):
    """read-only and read : write streams over a fresh (B, 2L) int32 buffer"""
    lib = ceiling_lib()
    st = torch.randint(-2, 3, (B, 2 * L), dtype=torch.int32, device=dev)
    out = torch.zeros(16384, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    nbytes = B * 8 * L
    res = {}
    # LDS per 4-wave block: 40 KB -> 4 blocks per CU = 4 waves/SIMD (the L = 128 step's occupancy);
    # 20 KB -> 8 waves/SIMD
    cases = [("read_grid", 0, 8, 1024)]
    for nb in (8, 16):
        for kind, name in ((1, "read_tile"), (2, "read_tile_pipe"), (3, "rw_tile"), (4, "rw_tile_pipe")):
            for lds, occ in ((40 * 1024, 4), (20 * 1024, 8)):
                cases.append((f"{name}_nb{nb}_occ{occ}", kind, nb, lds))
    for name, kind, nb, lds in cases:
        ts = []
        for r in range(reps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rc = lib.probe_run(kind, nb, st.data_ptr(), B, L, lds, out.data_ptr(), s)
            e1.record()
            torch.cuda.synchronize()
            assert rc == 0, (name, rc)
            if r:
                ts.append(e0.elapsed_time(e1))
        med = statistics.median(ts)
        moved = nbytes * (1.25 if kind in (3, 4) else 1.0)
        res[name] = {"median_ms": round(med, 4), "TB_s": round(moved / (med * 1e-3) / 1e12, 3),
                     "frac": round(moved / (med * 1e-3) / 1e9 / PEAK, 4)}
    del st, out
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="*")
    ap.add_argument("--L", type=int, default=128)
    ap.add_argument("--B", type=int, default=1 << 20)
    ap.add_argument("--K", type=int, default=20)
    ap.add_argument("--W", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--ceiling", action="store_true")
    a = ap.parse_args()
    L, B, K, W, H = a.L, a.B, a.K, a.W, 200
    dev = torch.device("cuda:0")
    out = {"L": L, "B": B, "K": K}
    if a.ceiling:
        out["ceilings"] = ceilings(L, B, a.reps, dev)
    libs = []
    for p in a.libs:
        path, _, mode = p.partition("@")
        libs.append((os.path.basename(path) + (f"@{mode}" if mode else ""), (load(path), mode or "full")))
    if libs:
        starts = torch.as_tensor(ms_starts(L, B)).to(dev)
        g = torch.Generator(device=dev)
        g.manual_seed(0)
        acts = torch.randint(0, 12, (W + K + 8, B), dtype=torch.int32, device=dev, generator=g)
        st = torch.empty_like(starts)
        cnt = torch.zeros(B, dtype=torch.int32, device=dev)
        rew = torch.empty(B, dtype=torch.int32, device=dev)
        dn = torch.empty(B, dtype=torch.uint8, device=dev)
        tr = torch.empty(B, dtype=torch.uint8, device=dev)
        lens = torch.empty((B, 2), dtype=torch.int32, device=dev)
        err = torch.zeros(B, dtype=torch.uint8, device=dev)
        red = torch.zeros(B, dtype=torch.uint8, device=dev)
        ec = torch.zeros(1, dtype=torch.int32, device=dev)
        s = torch.cuda.current_stream().cuda_stream

        def step(lm, t):
            lib, mode = lm
            if mode == "full":
                rc = lib.acx_step(st.data_ptr(), st.data_ptr(), acts[t].data_ptr(), starts.data_ptr(), cnt.data_ptr(),
                                  rew.data_ptr(), dn.data_ptr(), tr.data_ptr(), lens.data_ptr(), None, err.data_ptr(),
                                  ec.data_ptr(), B, L, H, 1, s)
            elif mode == "reduced":
                rc = lib.acx_step_lengths_reduced(st.data_ptr(), acts[t].data_ptr(), starts.data_ptr(), cnt.data_ptr(),
                                                  rew.data_ptr(), dn.data_ptr(), tr.data_ptr(), lens.data_ptr(),
                                                  red.data_ptr(), None, err.data_ptr(), ec.data_ptr(), B, L, H, 1, s)
            else:
                if mode == "LL":
                    lens.fill_(L)
                rc = lib.acx_step_lengths(st.data_ptr(), acts[t].data_ptr(), starts.data_ptr(), cnt.data_ptr(),
                                          rew.data_ptr(), dn.data_ptr(), tr.data_ptr(), lens.data_ptr(), None,
                                          err.data_ptr(), ec.data_ptr(), B, L, H, 1, s)
            assert rc == 0, rc

        ms = {n: [] for n, _ in libs}
        ref = None
        chg = None
        for rep in range(a.reps + 1):
            for n, lib in libs:
                st.copy_(starts)
                cnt.zero_()
                ec.zero_()
                red.zero_()
                nz = st.view(B, 2, L) != 0
                lens.copy_((nz * torch.arange(1, L + 1, device=dev, dtype=torch.int32)).amax(2))
                for t in range(W):
                    step(lib, t)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for t in range(W, W + K):
                    step(lib, t)
                e1.record()
                torch.cuda.synchronize()
                if rep:
                    ms[n].append(e0.elapsed_time(e1) / K)
                sig = (int(st.sum(dtype=torch.int64)), int((st * st).sum(dtype=torch.int64)),
                       int(cnt.sum(dtype=torch.int64)), int(rew.sum(dtype=torch.int64)), int(ec.item()))
                ref = ref or sig
                if os.environ.get("AB_NOCHECK") != "1":  # 1: diagnostic builds whose results differ on purpose
                    assert sig == ref, (n, sig, ref)
                if chg is None:
                    c = 0.0
                    for t in range(W + K, W + K + 8):
                        before = st.clone()
                        step(lib, t)
                        c += float((before.view(B, 2, L) != st.view(B, 2, L)).any(2).sum().item()) / B
                    chg = c / 8
        # the (L, L) refill alone (the LL entries' per-call extra launch)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(K):
            lens.fill_(L)
        e1.record()
        torch.cuda.synchronize()
        out["LL_refill_ms"] = round(e0.elapsed_time(e1) / K, 4)
        sb = 8 * L + 27 + 4 * L * chg
        out["changed_relators_per_env_step"] = chg
        out["bytes_per_env_step"] = sb
        for n, v in ms.items():
            med = statistics.median(v)
            out[n] = {"median_ms_per_step": round(med, 4), "min": round(min(v), 4), "all": [round(x, 4) for x in v],
                      "frac": round(B * sb / (med * 1e-3) / 1e9 / PEAK, 4)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
