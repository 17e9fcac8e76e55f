"""Where a launch of the rollout's store pattern spends its time (tools/timeline_probe.hip):
per-block start / end clocks, XCC, and per-step clocks of each block's wave 0, for K-step
launches at B = 2^20, L = 36.  The store pattern alone costs ~0.23 ms + 43 us per step
(profiles/r05/r05zza_store_k*.json): this shows whether the fixed part is the ramp after the
launch, the hand-over between the two resident rounds, or the tail.

    python tools/timeline_probe.py [--K 20,200]
"""
import argparse
import ctypes
import json
import os
import subprocess

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def lib():
    so = os.path.join(HERE, "libtimeline_probe.so")
    src = os.path.join(HERE, "timeline_probe.hip")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.check_call(["hipcc", "-O3", "--offload-arch=gfx950", "-shared", "-fPIC", src, "-o", so])
    L = ctypes.CDLL(so)
    L.timeline_tile.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    return L


def q(x, ps=(0, 10, 50, 90, 100)):
    if len(x) == 0:
        return {}
    return {f"p{p}": round(float(np.percentile(x, p)), 2) for p in ps}


def analyse(rec, steps, K, ev_ms, kind):
    st, en, xcc = rec[:, 0].astype(np.float64), rec[:, 1].astype(np.float64), rec[:, 2]
    ntile = rec[:, 3]
    t0 = st.min()
    st, en = (st - t0) / 100.0, (en - t0) / 100.0  # 100 MHz clock -> us
    stp = (steps.astype(np.float64) - t0) / 100.0
    span = en.max()
    order = np.argsort(st, kind="stable")
    nb = len(st)
    res = {"kind": KINDS[kind], "K": K, "event_ms": round(ev_ms, 4), "span_us": round(span, 1), "blocks": nb,
           "start_us": q(st), "end_us": q(en), "duration_us": q(en - st)}
    # the two rounds: blocks that start before the first block ends are the first round
    first_end = en.min()
    r1 = st < first_end
    res["round1_blocks"] = int(r1.sum())
    res["round1"] = {"start_us": q(st[r1]), "end_us": q(en[r1]), "duration_us": q(en[r1] - st[r1])}
    res["round2"] = {"start_us": q(st[~r1]), "end_us": q(en[~r1]), "duration_us": q(en[~r1] - st[~r1])}
    # per-step time of wave 0 inside a block: step t's start minus step t-1's, over all blocks
    if K > 1:
        d = np.diff(stp, axis=1)
        res["step_us_by_step"] = [round(float(np.median(d[:, t])), 2) for t in range(K - 1)]
        res["first_step_after_start_us"] = q(stp[:, 0] - st)
        res["last_step_to_end_us"] = q(en - stp[:, -1])
    # active blocks over time, 40 bins
    bins = np.linspace(0, span, 41)
    act = [int(((st < bins[i + 1]) & (en > bins[i])).sum()) for i in range(40)]
    res["active_blocks_by_bin"] = act
    res["bin_us"] = round(span / 40, 2)
    res["xcc"] = {int(x): {"blocks": int((xcc == x).sum()), "max_end_us": round(float(en[xcc == x].max()), 1),
                           "median_duration_us": round(float(np.median((en - st)[xcc == x])), 1),
                           "tiles": int(ntile[xcc == x].sum()) if kind else int((xcc == x).sum())}
                  for x in np.unique(xcc)}
    res["xcc_equals_block_mod_8"] = bool(np.all(xcc == (np.arange(nb) % 8)))
    return res


KINDS = ["block_per_tile", "persistent_dynamic", "persistent_static", "block_per_tile_xcc_weighted", "block_per_ticket",
         "block_per_tile_prio"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", default="20,200")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--kinds", default="0,1,2")
    ap.add_argument("--per-cu", default="8", help="persistent blocks per CU (4 waves each), comma-separated")
    ap.add_argument("--odd-pct", default="100,78", help="kind 3: an odd XCC's tiles as a percentage of an even one's")
    ap.add_argument("--over", default="100,125", help="kind 4: blocks launched as a percentage of the tiles")
    ap.add_argument("--prio", default="1,2,3", help="kind 5: priority modes (1 by progress, 2 young first, 3 fixed)")
    a = ap.parse_args()
    P = lib()
    dev = torch.device("cuda:0")
    B, L = 1 << 20, 36
    out = []
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    ctr = torch.zeros(4, dtype=torch.int32, device=dev)
    for K in [int(k) for k in a.K.split(",")]:
        obs = torch.zeros((K, B, 2 * L), dtype=torch.int32, device=dev)
        s = torch.cuda.current_stream().cuda_stream
        runs = [(int(k), int(p)) for k in a.kinds.split(",")
                for p in ({"0": ["8"], "3": a.odd_pct.split(","), "4": a.over.split(","), "5": a.prio.split(",")}.get(k) or a.per_cu.split(","))]
        for kind, per_cu in runs:
            grid = ncu * per_cu if kind in (1, 2) else per_cu  # persistent: per_cu waves per SIMD; else the kind's parameter
            nb = B // 256 if kind in (0, 3, 4, 5) else grid
            rec = torch.zeros((nb, 4), dtype=torch.int64, device=dev)
            steps = torch.zeros((nb, K), dtype=torch.int64, device=dev)
            ms = []
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                rc = P.timeline_tile(kind, obs.data_ptr(), B, L, K, grid, ctr.data_ptr(), rec.data_ptr(),
                                     steps.data_ptr(), s)
                assert rc == 0, rc
                e1.record()
                torch.cuda.synchronize()
                ms.append(e0.elapsed_time(e1))
            r = analyse(rec.cpu().numpy().view(np.uint64), steps.cpu().numpy().view(np.uint64), K, ms[-1], kind)
            r["event_ms_all"] = [round(m, 4) for m in ms]
            r["blocks_per_cu" if kind in (1, 2) else "param"] = per_cu
            if kind == 4:
                assert int(ctr[0].item()) == 0 and int(ctr[1].item()) == 0, "ticket counters not reset"
            r["TBps"] = round(obs.numel() * 4 / (min(ms[1:] or ms) * 1e-3) / 1e12, 3)
            out.append(r)
            print(json.dumps(r), flush=True)
        del obs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
