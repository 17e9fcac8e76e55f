"""In-process A/B of greedy builds: acx_greedy_run from AK(3) (L = 36, cyclical = False) and a
Miller-Schupp start, to 10^6 nodes, through each library in turn, REPS rounds interleaved; wall
time of the C call, the engine's own split (GPU round trips / host replay / selection), and the
popped-parent and node counts, which must agree between the libraries (same search).

    python tools/ab_greedy.py abv/libacx_base.so ac-solver-caltech_amd/acx/libacx.so [--reps 5]

A library here is a whole libacx.so (tools/ab_build.sh builds only the env-step kernels):
`ab_greedy_build.sh`-style, e.g. `git show REV:ac-solver-caltech_amd/csrc/acx_greedy.hip` built
with build.py's flags into another directory."""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ac-solver-caltech_amd"))
P, I32, I64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64


def load(path):
    lib = ctypes.CDLL(os.path.abspath(path))
    lib.acx_greedy_run.argtypes = [P, I32, I64, I32, I32, P]
    lib.acx_greedy_run.restype = ctypes.c_int
    lib.acx_greedy_stats.argtypes = [P, P]
    lib.acx_greedy_status.argtypes = [P, P, P, P]
    lib.acx_greedy_status.restype = I32
    lib.acx_greedy_destroy.argtypes = [P]
    return lib


def run(lib, pres, L, budget):
    h = ctypes.c_void_p(0)
    t0 = time.perf_counter()
    st = lib.acx_greedy_run(pres.ctypes.data, L, budget, 0, 0, ctypes.byref(h))
    wall = time.perf_counter() - t0
    assert st == 0, st
    s = np.zeros(13, np.int64)
    lib.acx_greedy_stats(h, s.ctypes.data)
    b, m, n = I32(0), I32(0), I64(0)
    status = lib.acx_greedy_status(h, ctypes.byref(b), ctypes.byref(m), ctypes.byref(n))
    lib.acx_greedy_destroy(h)
    return wall, {"rounds": int(s[0]), "expanded": int(s[1]), "pops": int(s[2]), "nodes": int(n.value),
                  "status": int(status), "gpu_s": s[5] / 1e9, "replay_s": s[6] / 1e9, "select_s": s[4] / 1e9}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--budget", type=int, default=10 ** 6)
    a = ap.parse_args()
    torch.zeros(1, device="cuda")  # the HIP runtime up before the libraries are used
    from acx.data import load_initial_states
    from acx.envs.utils import convert_relators_to_presentation

    L = 36
    cases = {"AK3": convert_relators_to_presentation([1, 1, 1, -2, -2, -2, -2], [1, 2, 1, -2, -1, -2], L),
             "MS700": load_initial_states("all", L)[700]}
    cases = {k: np.ascontiguousarray(v, dtype=np.int32) for k, v in cases.items()}
    libs = [(os.path.basename(os.path.dirname(p)) + "/" + os.path.basename(p), load(p)) for p in a.libs]
    res = {(n, c): [] for n, _ in libs for c in cases}
    last = {}
    for rep in range(a.reps + 1):
        for n, lib in libs:
            for c, pres in cases.items():
                wall, st = run(lib, pres, L, a.budget)
                key = (st["pops"], st["nodes"], st["status"])
                assert last.setdefault(c, key) == key, (c, n, key, last[c])
                if rep:
                    res[(n, c)].append((wall, st))
    out = {"what": "tools/ab_greedy.py: acx_greedy_run to %d nodes, medians of %d interleaved runs" % (a.budget, a.reps),
           "cases": {}}
    for (n, c), v in res.items():
        med = lambda f: statistics.median(f(x) for x in v)  # noqa: E731
        out["cases"][f"{n} {c}"] = {"wall_ms": round(med(lambda x: x[0]) * 1e3, 2),
                                    "gpu_ms": round(med(lambda x: x[1]["gpu_s"]) * 1e3, 2),
                                    "replay_ms": round(med(lambda x: x[1]["replay_s"]) * 1e3, 2),
                                    "select_ms": round(med(lambda x: x[1]["select_s"]) * 1e3, 2),
                                    "pops": v[0][1]["pops"], "nodes": v[0][1]["nodes"], "rounds": v[0][1]["rounds"]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
