"""Same-box A/B of owner-partitioned BFS builds: AK(3), L = 36, to NODES nodes at one rank, each
library (a whole libacx.so, e.g. a build of an earlier revision) in its own process via ACX_LIB,
the processes interleaved ROUNDS times; per process a warmup then REPS timed searches (wall clock
around the call, after a synchronize), plus the device BFS in the same process for scale.

    python tools/ab_sbfs.py abv/libacx_r03.so:abv/r03/ac-solver-caltech_amd ac-solver-caltech_amd/acx/libacx.so

Each entry is LIB or LIB:PKGROOT -- the Python package (acx) the library is driven by, e.g. an
earlier revision's (`git archive REV ac-solver-caltech_amd/acx | tar -x -C DIR`), whose C-ABI
calls match that library's.  [--nodes 1e7] [--rounds 3] [--reps 5]
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)

CHILD = r"""
import contextlib, io, json, sys, time
sys.path.insert(0, %(pkg)r)
import torch
from acx.envs.utils import convert_relators_to_presentation
from acx.search import _sharded_bfs as S, _device_bfs as D
dev = torch.device("cuda:0")
ak3 = convert_relators_to_presentation([1, 1, 1, -2, -2, -2, -2], [1, 2, 1, -2, -1, -2], 36)
n = int(float(%(nodes)r))
out = {}
for name, fn in (("sharded", lambda: S.sharded_bfs(ak3, n, device=dev)), ("device", lambda: D.device_bfs(ak3, n, device=dev))):
    ts = []
    for r in range(%(reps)d + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with contextlib.redirect_stdout(io.StringIO()):
            fn()
        torch.cuda.synchronize()
        if r:
            ts.append((time.perf_counter() - t0) * 1e3)
    out[name] = ts
print(json.dumps(out))
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--nodes", default="1e7")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    res = {lib: {"sharded": [], "device": []} for lib in a.libs}
    for _ in range(a.rounds):
        for entry in a.libs:
            lib, _, pkg = entry.partition(":")
            code = CHILD % {"pkg": os.path.abspath(pkg or os.path.join(REPO, "ac-solver-caltech_amd")),
                            "nodes": a.nodes, "reps": a.reps}
            env = dict(os.environ, ACX_LIB=os.path.abspath(lib))
            p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=300)
            if p.returncode != 0:
                sys.exit(f"{entry}: {p.stderr[-2000:]}")
            d = json.loads(p.stdout.strip().splitlines()[-1])
            for k in d:
                res[entry][k] += d[k]
    out = {"nodes": a.nodes, "rounds": a.rounds, "reps_per_process": a.reps}
    for lib, d in res.items():
        out[os.path.basename(lib.partition(":")[0]) if "abv" in lib else lib] = {
            k: {"median_ms": round(statistics.median(v), 4), "min_ms": round(min(v), 4), "all": [round(x, 4) for x in v]}
            for k, v in d.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
