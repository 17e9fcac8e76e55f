"""Summarise tools/profile_rollout_sq.sh output into <out>/<tag>_rollout_sq_summary.json: for the
timed (last) dispatch of each rollout kernel (int32 obs: rollout_kernel<..,1>, int8 obs: <..,2>)
the SQ counters totalled over the chip, per wave-step (16,384 waves x K steps at 2^20 envs) and
the kernel's duration from the trace pass.

    python tools/summarize_rollout_sq.py gpurun_out/prof_rsq_<tag> <tag> profiles/<round> [K]"""
import collections
import csv
import json
import os
import sys

d, tag, out = sys.argv[1], sys.argv[2], sys.argv[3]
K = int(sys.argv[4]) if len(sys.argv) > 4 else 20
res = {"tag": tag, "steps": K, "kernels": {}}


def short(n):
    return n.split("(")[0].replace("void ", "")


for kind in ("pmc_sq", "pmc_sq2"):
    p = os.path.join(d, kind, "r_counter_collection.csv")
    last = {}
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    with open(p) as f:
        for r in csv.DictReader(f):
            if "rollout_kernel" not in r["Kernel_Name"]:
                continue
            k, disp = short(r["Kernel_Name"]), int(r["Dispatch_Id"])
            vals[(k, disp)][r["Counter_Name"]] += float(r["Counter_Value"])
            last[k] = max(last.get(k, -1), disp)
    for k, disp in last.items():
        e = res["kernels"].setdefault(k, {})
        c = vals[(k, disp)]
        waves = c.get("SQ_WAVES") or e.get("SQ_WAVES") or 16384.0
        for name, v in c.items():
            e[name] = v
            if name not in ("SQ_WAVES",):
                e[name + "_per_wave_step"] = v / waves / K
with open(os.path.join(d, "trace", "r_kernel_stats.csv")) as f:
    for r in csv.DictReader(f):
        k = short(r["Name"])
        if k in res["kernels"]:
            res["kernels"][k]["max_dispatch_us"] = float(r["MaxNs"]) / 1e3
os.makedirs(out, exist_ok=True)
with open(os.path.join(out, f"{tag}_rollout_sq_summary.json"), "w") as f:
    json.dump(res, f, indent=1)
print(json.dumps({k: {n: round(v, 1) for n, v in e.items() if n.endswith("per_wave_step") or n == "max_dispatch_us"}
                  for k, e in res["kernels"].items()}, indent=1))
