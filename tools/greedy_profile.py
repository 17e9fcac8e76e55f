"""Where the device greedy search's time goes (csrc/acx_greedy.hip engine statistics): greedy_search
from AK(3), L = 36, cyclical = False, to 10^6 nodes (BASELINE configs[3], greedy half), for a few
expansion batch sizes; best of REPS wall times after a warm-up.

    python tools/greedy_profile.py [--batch 256,512,1024] [--nodes 1000000] [--reps 2]
"""
import argparse
import contextlib
import io
import json
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "ac-solver-caltech_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", default="0")
    ap.add_argument("--nodes", type=int, default=10 ** 6)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    from acx.envs.utils import convert_relators_to_presentation
    from acx.search import _engine as E
    from acx.search import greedy_search

    dev = torch.device("cuda:0")
    ak3 = convert_relators_to_presentation([1, 1, 1, -2, -2, -2, -2], [1, 2, 1, -2, -1, -2], 36)
    for b in [int(x) for x in a.batch.split(",")]:
        with contextlib.redirect_stdout(io.StringIO()):
            greedy_search(ak3, a.nodes, device=dev, batch=b or None)
        best, st, res = None, None, None
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            with contextlib.redirect_stdout(io.StringIO()):
                r = greedy_search(ak3, a.nodes, device=dev, batch=b or None)
            w = time.perf_counter() - t0
            if best is None or w < best:
                best, st, res = w, {k: v for k, v in E.LAST_STATS.items() if k not in ("min_trace",)}, r
        st = {k: (round(v * 1e3, 3) if k.endswith("_s") else v) for k, v in st.items()}
        print(json.dumps({"batch": b, "wall_ms": round(best * 1e3, 2), "path_len": len(res[1]), "found": bool(res[0]),
                          "stats_ms_for_*_s": st}), flush=True)


if __name__ == "__main__":
    main()
