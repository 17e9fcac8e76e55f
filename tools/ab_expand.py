"""In-process A/B of expand12 builds (tools/ab_build.sh): acx_expand12 with full int32 children
(+ lengths, no keys), or with --keys the packed child keys only (config 4's expansion), over N parents (Miller-Schupp starts at L = 36), each library in turn on the
SAME buffers, REPS rounds interleaved, HIP events; every library must write the same children.

    python tools/ab_expand.py abv/libacx_a.so abv/libacx_b.so ... [--N 1000000] [--reps 5]
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

P, I32, I64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--N", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--keys", action="store_true")
    a = ap.parse_args()
    L, N = 36, a.N
    dev = torch.device("cuda:0")
    libs = []
    for p in a.libs:
        lib = ctypes.CDLL(os.path.abspath(p))
        lib.acx_expand12.argtypes = [P] * 6 + [I64, I32, I32, P]
        libs.append((os.path.basename(p), lib))
    par = torch.as_tensor(ms_starts(L, N)).to(dev)
    kw = (4 * L + 16 + 63) // 64
    if a.keys:
        ch = torch.empty((N, 12, kw), dtype=torch.int64, device=dev)
        ln = None
    else:
        ch = torch.empty((N, 12, 2 * L), dtype=torch.int32, device=dev)
        ln = torch.empty((N, 12, 2), dtype=torch.int32, device=dev)
    ms = {n: [] for n, _ in libs}
    ref = None
    for rep in range(a.reps + 1):
        for n, lib in libs:
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            if a.keys:
                rc = lib.acx_expand12(par.data_ptr(), None, None, ch.data_ptr(), None, None, N, L, 0,
                                      torch.cuda.current_stream().cuda_stream)
            else:
                rc = lib.acx_expand12(par.data_ptr(), ch.data_ptr(), ln.data_ptr(), None, None, None, N, L, 0,
                                      torch.cuda.current_stream().cuda_stream)
            e1.record()
            torch.cuda.synchronize()
            assert rc == 0, rc
            if rep == 0:
                cs = int(ch.sum(dtype=torch.int64).item()) ^ int((ch * 7 + 1).sum(dtype=torch.int64).item())
                ref = cs if ref is None else ref
                assert cs == ref, n
            else:
                ms[n].append(e0.elapsed_time(e1))
    bpp = 8 * L + 12 * kw * 8 if a.keys else 8 * L + 12 * (8 * L + 8)
    out = {"N": N, "bytes_per_parent": bpp, "libs": {}}
    for n, v in ms.items():
        m = statistics.median(v)
        out["libs"][n] = {"median_ms": round(m, 4), "frac": round(N * bpp / (m * 1e-3) / 1e9 / 8000, 4), "all": v}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
