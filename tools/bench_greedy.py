"""greedy_search / bfs throughput on the GPU path (acx) for a few presentations and budgets.

    python tools/bench_greedy.py [budget]

Reports wall time, nodes discovered and parents popped per second.  The reference's
CPU greedy_search pops ~1.8k parents/s (SURVEY.md §6, 12 ACMove calls per pop)."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ac-solver-caltech_amd"))
import acx  # noqa: E402
from acx.envs.utils import convert_relators_to_presentation  # noqa: E402

budget = int(sys.argv[1]) if len(sys.argv) > 1 else 10 ** 6
cases = {
    "AK3_L36": convert_relators_to_presentation([1, 1, 1, -2, -2, -2, -2], [1, 2, 1, -2, -1, -2], 36),
    "MS_idx700_L36": acx.data.load_initial_states("all", 36)[700],
}
out = {}
for name, p in cases.items():
    for fn in (acx.greedy_search, acx.bfs):
        t0 = time.perf_counter()
        ok, path = fn(presentation=p, max_nodes_to_explore=budget)
        dt = time.perf_counter() - t0
        from acx.search import _device_bfs, _engine
        stats = _device_bfs.LAST_STATS if fn is acx.bfs else _engine.LAST_STATS
        out[f"{fn.__name__}_{name}"] = {"solved": bool(ok), "path_len": len(path) if path else None,
                                       "budget": budget, "wall_s": dt, "nodes_per_s": budget / dt,
                                       **{k: v for k, v in stats.items() if k != "node_keys"}}
print(json.dumps(out, indent=1))
