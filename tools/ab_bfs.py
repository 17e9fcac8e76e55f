"""A/B of device-BFS library builds (e.g. a -D variant of acx_bfs.hip linked with the other
objects): each library in its own process (ACX_LIB), the processes interleaved ROUNDS times on
one box; per process the device BFS from AK(3) (config 4) to each budget, best of 5 after a
warm-up, with the node count and status (which must agree across libraries).

    python tools/ab_bfs.py lib1.so lib2.so ... [--budgets 1e7,1e8] [--rounds 2]
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def worker(budgets):
    sys.path.insert(0, os.path.join(REPO, "ac-solver-caltech_amd"))
    import torch
    from acx.envs.utils import convert_relators_to_presentation
    from acx.search import _device_bfs as D
    dev = torch.device("cuda:0")
    ak3 = convert_relators_to_presentation([1, 1, 1, -2, -2, -2, -2], [1, 2, 1, -2, -1, -2], 36)
    out = {}
    for nb in budgets:
        D.device_bfs(ak3, nb, device=dev)
        walls = []
        for _ in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            D.device_bfs(ak3, nb, device=dev)
            walls.append((time.perf_counter() - t0) * 1e3)
        out[str(nb)] = {"best_ms": min(walls), "walls_ms": walls, "nodes": D.LAST_STATS["nodes"],
                        "status": D.LAST_STATS["status"]}
        D.release_workspaces()
    print(json.dumps(out))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="*")
    ap.add_argument("--budgets", default="1e7,1e8")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--worker", action="store_true")
    a = ap.parse_args()
    budgets = [int(float(x)) for x in a.budgets.split(",")]
    if a.worker:
        worker(budgets)
        return
    res = {os.path.basename(l): [] for l in a.libs}
    for r in range(a.rounds):
        for lib in a.libs:
            env = dict(os.environ, ACX_LIB=os.path.abspath(lib))
            p = subprocess.run([sys.executable, os.path.abspath(__file__), "--worker", "--budgets", a.budgets],
                               env=env, capture_output=True, text=True, timeout=600)
            if p.returncode != 0:
                print(p.stderr[-3000:], file=sys.stderr)
                sys.exit(p.returncode)
            res[os.path.basename(lib)].append(json.loads(p.stdout.strip().splitlines()[-1]))
            print(f"round {r} {lib} done", file=sys.stderr, flush=True)
    summary = {lib: {b: min(run[b]["best_ms"] for run in runs) for b in runs[0]} for lib, runs in res.items()}
    print(json.dumps({"best_ms": summary, "runs": res}))


if __name__ == "__main__":
    main()
