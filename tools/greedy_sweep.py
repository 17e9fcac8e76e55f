"""greedy_search (device visited-set engine) on AK(3), L = 36, 10^6 nodes at several round sizes
(parents expanded per GPU round): wall time and the engine's round statistics, second of two
runs each.

    python tools/greedy_sweep.py [batch,...] [budget]"""
import contextlib
import io
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ac-solver-caltech_amd"))
import acx  # noqa: E402
from acx.envs.utils import convert_relators_to_presentation  # noqa: E402
from acx.search import _engine  # noqa: E402

batches = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [32, 64, 128, 256, 512]
budget = int(float(sys.argv[2])) if len(sys.argv) > 2 else 10 ** 6
cases = {"AK3": convert_relators_to_presentation([1, 1, 1, -2, -2, -2, -2], [1, 2, 1, -2, -1, -2], 36),
         "MS700": acx.data.load_initial_states("all", 36)[700]}
out = {}
for name, p in cases.items():
    for b in batches:
        for rep in range(2):
            t0 = time.perf_counter()
            with contextlib.redirect_stdout(io.StringIO()):
                ok, path = acx.greedy_search(presentation=p, max_nodes_to_explore=budget, batch=b)
            dt = time.perf_counter() - t0
        st = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in _engine.LAST_STATS.items()
              if k not in ("node_keys", "min_trace", "popped")}
        out[f"{name}_b{b}"] = {"wall_s": round(dt, 4), "path_len": len(path), **st}
        print(json.dumps({f"{name}_b{b}": out[f"{name}_b{b}"]}), file=sys.stderr, flush=True)
    # the host-dedup engine (round 1's path: acx_expand12 launches + csrc/acx_search.cpp), warm
    for rep in range(2):
        t0 = time.perf_counter()
        with contextlib.redirect_stdout(io.StringIO()):
            ok, path = acx.greedy_search(presentation=p, max_nodes_to_explore=budget, engine="host")
        dt = time.perf_counter() - t0
    st = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in _engine.LAST_STATS.items()
          if k not in ("node_keys", "min_trace", "popped")}
    out[f"{name}_host"] = {"wall_s": round(dt, 4), "path_len": len(path), **st}
    print(json.dumps({f"{name}_host": out[f"{name}_host"]}), file=sys.stderr, flush=True)
print(json.dumps(out))
