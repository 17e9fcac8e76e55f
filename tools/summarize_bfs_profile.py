"""Summarise tools/profile_bfs.sh output (rocprofv3 over tools/bench_bfs.py 1e7) into
profiles/<round>/<tag>_bfs_summary.json: per acx kernel the dispatch count, mean duration, and the
mean per-dispatch PMC values (FETCH_SIZE / WRITE_SIZE in bytes -- FETCH_SIZE NOT doubled: these
kernels' reads are 8-16 B gathers, not the wide streams the gfx950 correction is for -- the SQ
instruction / wait counters, TCC hits and misses), plus the bench JSON of the un-profiled run.

    python tools/summarize_bfs_profile.py gpurun_out/prof_bfs_<tag> <tag> profiles/<round>"""
import collections
import csv
import json
import os
import shutil
import sys

d, tag, out_dir = sys.argv[1], sys.argv[2], sys.argv[3]
os.makedirs(out_dir, exist_ok=True)


def short(n):
    return n.split("(")[0].replace("void ", "")


res = {"tag": tag, "kernels": {}}
with open(os.path.join(d, "trace", "bfs_kernel_stats.csv")) as f:
    for r in csv.DictReader(f):
        if "acx" not in r["Name"]:
            continue
        res["kernels"][short(r["Name"])] = {"dispatches": int(r["Calls"]), "mean_us": float(r["AverageNs"]) / 1e3,
                                           "total_ms": float(r["TotalDurationNs"]) / 1e6}
for kind in ("pmc_fetch", "pmc_write", "pmc_sq", "pmc_tcc"):
    p = os.path.join(d, kind, "bfs_counter_collection.csv")
    if not os.path.exists(p):
        continue
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    with open(p) as f:
        for r in csv.DictReader(f):
            if "acx" in r["Kernel_Name"]:
                agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in agg.items():
        e = res["kernels"].setdefault(k, {})
        for c, v in cs.items():
            scale = 1024 if c in ("FETCH_SIZE", "WRITE_SIZE") else 1
            e[c + ("_bytes" if scale == 1024 else "") + "_per_dispatch"] = sum(v) / len(v) * scale
for k, e in res["kernels"].items():
    if "SQ_WAIT_ANY_per_dispatch" in e and e.get("SQ_WAVE_CYCLES_per_dispatch"):
        e["wait_frac_of_wave_cycles"] = e["SQ_WAIT_ANY_per_dispatch"] / e["SQ_WAVE_CYCLES_per_dispatch"]
    h, m = e.get("TCC_HIT_sum_per_dispatch"), e.get("TCC_MISS_sum_per_dispatch")
    if h is not None and m:
        e["tcc_hit_rate"] = h / (h + m)
bj = os.path.join(d, "bench.json")
if os.path.exists(bj):
    for line in open(bj):
        if line.startswith("{"):
            res["bench"] = json.loads(line)
with open(os.path.join(out_dir, f"{tag}_bfs_summary.json"), "w") as f:
    json.dump(res, f, indent=1)
shutil.copy(os.path.join(d, "trace", "bfs_kernel_stats.csv"), os.path.join(out_dir, f"{tag}_bfs_kernel_stats.csv"))
print(json.dumps({k: {a: round(b, 3) for a, b in v.items()} for k, v in res["kernels"].items()}, indent=0)[:3000])
