"""Summarise a rocprofv3 run of bench.py (profile_cmd.sh output) into profiles/<tag>_summary.json.

Reads <dir>/trace/bench_kernel_stats.csv, <dir>/trace/bench_kernel_trace.csv,
<dir>/pmc_fetch/bench_counter_collection.csv, <dir>/pmc_write/bench_counter_collection.csv
and <dir>/trace_bench.log (the bench JSON line printed under the profiler).

HBM traffic per dispatch follows MI355X_MICROARCH.md "HBM": FETCH_SIZE / WRITE_SIZE are in
KiB; FETCH_SIZE reads exactly half of a wide coalesced streaming read on gfx950, so it is
doubled before comparing with a byte count; WRITE_SIZE is exact for 16-B-per-lane stores."""
import csv
import gzip
import json
import os
import shutil
import sys

d, tag = sys.argv[1], sys.argv[2]
out_dir = sys.argv[3] if len(sys.argv) > 3 else "profiles"
os.makedirs(out_dir, exist_ok=True)


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


trace = sorted(rows(os.path.join(d, "trace", "bench_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
disp = {}
starts = {}
for r in trace:
    name = r["Kernel_Name"]
    if "acx::" not in name:
        continue
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    disp.setdefault(name, []).append(dur)
    starts.setdefault(name, []).append(int(r["Start_Timestamp"]))
pmc = {}
for kind in ("fetch", "write"):
    p = os.path.join(d, f"pmc_{kind}", "bench_counter_collection.csv")
    if not os.path.exists(p):
        continue
    for r in sorted(rows(p), key=lambda r: int(r["Dispatch_Id"])):
        if "acx::" not in r["Kernel_Name"]:
            continue
        pmc.setdefault(r["Kernel_Name"], {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
bench = None
log = os.path.join(d, "trace_bench.log")
if os.path.exists(log):
    for line in open(log):
        if line.startswith("{"):
            bench = json.loads(line)
summary = {"tag": tag, "kernels": {}}
for name, durs in disp.items():
    k = {"dispatches": len(durs), "durations_ms": durs, "max_ms": max(durs), "mean_ms": sum(durs) / len(durs)}
    c = pmc.get(name, {})
    if "FETCH_SIZE" in c:
        k["fetch_bytes_corrected"] = [2 * v * 1024 for v in c["FETCH_SIZE"]]
    if "WRITE_SIZE" in c:
        k["write_bytes"] = [v * 1024 for v in c["WRITE_SIZE"]]
    summary["kernels"][name] = k
if bench:
    summary["bench_line"] = bench
    rl = bench["roofline"]
    # the timed launch = the last (in time) of the longest rollout_kernel dispatches (the warmup
    # launch comes first) plus, when ops.rollout packed the move ids first, the matching
    # pack_actions_kernel dispatch (the last pack dispatch that started after the previous
    # rollout dispatch and before this one: short launches read the int32 ids directly,
    # ops.packs_actions, so the pack and rollout dispatch counts differ)
    # the int32-trajectory instantiation: rollout_kernel<NW, LC, VEC, 1, PK> (round 2's int8 mode is
    # OBS = 2; before it the parameter was `true`, and before the PK parameter it ended there)
    import re
    timed = [(n, v) for n, v in summary["kernels"].items()
             if re.search(r"rollout_kernel<\d+, \d+, \d+, (1|true)(, (true|false))?>", n)]
    packs = [n for n in summary["kernels"] if "pack_actions_kernel" in n]

    def hbm(k, i):
        if "write_bytes" not in k:
            return None
        return (k.get("fetch_bytes_corrected", [0] * (i + 1))[i] or 0) + (k["write_bytes"][i] or 0)

    # dispatch order (bench.py): the headline's warmup launches, its timed launches, then the
    # variants' (desync, done-heavy) -- so the timed launches are the ones right after the warmup's
    bl = bench
    T_buf = min(max(bl["steps"], bl["warmup"]), 200)
    n_warm = -(-bl["warmup"] // T_buf) if bl["warmup"] > 0 else 0
    n_timed = rl.get("launches", 1)
    if timed:
        kname, k = max(timed, key=lambda nv: nv[1]["dispatches"])
        idx = list(range(n_warm, n_warm + n_timed))
        ms = sum(k["durations_ms"][i] for i in idx)
        parts = [hbm(k, i) for i in idx]
        traffic = None if None in parts else sum(parts)
        rec = {"timed_dispatch_index": idx, "rollout_kernel_ms": ms, "rollout_kernel_hbm_bytes": traffic,
               "rollout_kernel_fetch_bytes": sum(k.get("fetch_bytes_corrected", [0] * (idx[-1] + 1))[i] for i in idx),
               "rollout_kernel_write_bytes": sum(k.get("write_bytes", [0] * (idx[-1] + 1))[i] for i in idx)}
        pidx = []
        if packs:
            pname = packs[0]
            ps_ = starts[pname]
            rs_ = starts[kname]
            for i in idx:
                lo = rs_[i - 1] if i > 0 else -1
                cand = [j for j, t in enumerate(ps_) if lo < t < rs_[i]]
                if cand:
                    pidx.append(cand[-1])
        if pidx:
            pk = summary["kernels"][pname]
            pms = sum(pk["durations_ms"][j] for j in pidx)
            ms += pms
            pparts = [hbm(pk, j) for j in pidx]
            pt = None if None in pparts else sum(pparts)
            traffic = None if traffic is None or pt is None else traffic + pt
            rec.update({"pack_dispatch_index": pidx, "pack_actions_kernel_ms": pms, "pack_actions_hbm_bytes": pt})
        rec.update({
            "rocprof_ms": ms, "bench_event_ms": rl["kernel_ms"],
            "agree_pct": 100 * abs(ms - rl["kernel_ms"]) / rl["kernel_ms"],
            "algorithmic_bytes": rl["launch_bytes"],
            "pmc_hbm_bytes": traffic,
        })
        summary["rollout_timed_dispatch"] = rec
if bench and "random-action stepping" in bench["config"]["workload"]:
    # bench.py --workload step: the headline is K per-call acx_step_lengths launches after W
    # warmup calls and K off-the-clock ones (the live-byte accounting); before round 4's
    # lengths-carrying step it was acx_step's (step_kernel<.., false>)
    import re
    pat = (r"step_lengths_kernel<\d+, \d+, \d+>" if "step_lengths_kernel" in bench["roofline"].get("kernel", "")
           else r"step_kernel<\d+, \d+, \d+, false>")
    steps = [(n, v) for n, v in summary["kernels"].items() if re.search(pat, n)]
    if steps:
        kname, k = max(steps, key=lambda nv: nv[1]["dispatches"])
        W, K = bench["warmup"], bench["steps"]
        # the lengths-carrying headline runs its K steps once off the clock (byte accounting)
        # before the timed K; a profile from before that change has W + K + 8 dispatches
        acct = K if "step_lengths_kernel" in kname and k["dispatches"] >= W + 2 * K else 0
        idx = list(range(W + acct, W + acct + K))
        ms = [k["durations_ms"][i] for i in idx]
        tb = [(k.get("fetch_bytes_corrected") or [None] * (W + K))[i] for i in idx]
        wb = [(k.get("write_bytes") or [None] * (W + K))[i] for i in idx]
        per = bench["roofline"]["launch_bytes"]
        rec = {"kernel": kname, "timed_dispatch_index": [idx[0], idx[-1]], "mean_ms": sum(ms) / K,
               "bench_event_ms_per_launch": bench["roofline"]["kernel_ms"] / K,
               "algorithmic_bytes_per_launch": per}
        if None not in tb and None not in wb:
            rec.update(fetch_bytes_per_launch=sum(tb) / K, write_bytes_per_launch=sum(wb) / K,
                       pmc_hbm_bytes_per_launch=(sum(tb) + sum(wb)) / K,
                       pmc_over_algorithmic=(sum(tb) + sum(wb)) / K / per)
        rec["agree_pct"] = 100 * abs(rec["mean_ms"] - rec["bench_event_ms_per_launch"]) / rec["bench_event_ms_per_launch"]
        summary["step_timed_dispatches"] = rec
        print(json.dumps(rec, indent=1))
with open(os.path.join(out_dir, f"{tag}_summary.json"), "w") as f:
    json.dump(summary, f, indent=1)
# the per-kernel stats as they are; the per-dispatch traces and counter dumps gzipped (the
# summary above holds what bench.py reads from them)
if os.path.exists(os.path.join(d, "trace/bench_kernel_stats.csv")):
    shutil.copy(os.path.join(d, "trace/bench_kernel_stats.csv"), os.path.join(out_dir, f"{tag}_kernel_stats.csv"))
for src, dst in (("trace/bench_kernel_trace.csv", "kernel_trace.csv.gz"),
                 ("pmc_fetch/bench_counter_collection.csv", "pmc_fetch.csv.gz"),
                 ("pmc_write/bench_counter_collection.csv", "pmc_write.csv.gz")):
    if os.path.exists(os.path.join(d, src)):
        with open(os.path.join(d, src), "rb") as fi, gzip.open(os.path.join(out_dir, f"{tag}_{dst}"), "wb") as fo:
            shutil.copyfileobj(fi, fo)
if bench:
    with open(os.path.join(out_dir, f"{tag}_bench_under_rocprof.json"), "w") as f:
        f.write(json.dumps(bench) + "\n")
print(json.dumps(summary.get("rollout_timed_dispatch"), indent=1))
