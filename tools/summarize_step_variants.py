"""Per-variant check of bench.py's step byte accounting against rocprofv3 PMC (VERDICT r04
item 1): for every in-place step variant of a profiled bench run (profile_cmd.sh output dir),
the mean HBM bytes per timed launch (FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md "HBM") next
to the line's bytes_per_env_step x B.

    python tools/summarize_step_variants.py DIR TAG OUTDIR

Dispatch order of bench.py (one kernel name each): step_api = W warmup + K untimed replay + K
timed acx_step launches, then (lengths variant: W + K + K of step_lengths_kernel), then the
hipGraph = K warm + K timed replays of acx_step's launches; learner_step = 1 + KL replay + KL
timed launches of the learner instantiation; config2 (rollout headline only) = W2 + K2 replay +
K2 timed + K2 warm + K2 timed graph launches of the small-batch kernel."""
import csv
import json
import os
import sys

d, tag = sys.argv[1], sys.argv[2]
out_dir = sys.argv[3] if len(sys.argv) > 3 else "profiles"


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def per_kernel(path, col):
    out = {}
    for r in sorted(rows(path), key=lambda r: int(r["Dispatch_Id"])):
        if "acx::" in r["Kernel_Name"] and r.get("Counter_Name", col) == col:
            out.setdefault(r["Kernel_Name"].split("(")[0].replace("void ", ""), []).append(float(r["Counter_Value"]))
    return out


fetch = per_kernel(os.path.join(d, "pmc_fetch", "bench_counter_collection.csv"), "FETCH_SIZE")
write = per_kernel(os.path.join(d, "pmc_write", "bench_counter_collection.csv"), "WRITE_SIZE")
trace = {}
for r in sorted(rows(os.path.join(d, "trace", "bench_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"])):
    if "acx::" in r["Kernel_Name"]:
        n = r["Kernel_Name"].split("(")[0].replace("void ", "")
        trace.setdefault(n, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
line = None
for ln in open(os.path.join(d, "trace_bench.log")):
    if ln.startswith("{"):
        line = json.loads(ln)
W, K = line["warmup"], line["steps"]
B = line["config"]["envs_per_gpu"]
v = line["variants"]


def check(name, kernel, idx, bpe, launches_note):
    k = kernel.replace(" ", "")
    kk = next((n for n in fetch if n.replace(" ", "") == k), None)
    if kk is None or max(idx) >= len(fetch[kk]) or max(idx) >= len(write.get(kk, [])):
        return {"variant": name, "kernel": kernel, "error": "dispatches not found", "have": len(fetch.get(kk, []))}
    f = sum(2 * 1024 * fetch[kk][i] for i in idx) / len(idx)
    w = sum(1024 * write[kk][i] for i in idx) / len(idx)
    alg = bpe * B
    ms = [trace[kk][i] for i in idx] if kk in trace and max(idx) < len(trace[kk]) else []
    return {"variant": name, "kernel": kernel, "dispatches": [idx[0], idx[-1]], "launches": launches_note,
            "pmc_fetch_bytes_per_launch": f, "pmc_write_bytes_per_launch": w, "pmc_bytes_per_launch": f + w,
            "algorithmic_bytes_per_launch": alg, "pmc_over_algorithmic": (f + w) / alg,
            "within_3pct": abs((f + w) / alg - 1) <= 0.03,
            "rocprof_mean_ms": sum(ms) / len(ms) if ms else None}


res = []
if "step_api" in v:
    kn = v["step_api"]["roofline"]["kernel"].replace("acx::", "acx::")
    res.append(check("step_api", kn, list(range(W + K, W + 2 * K)), v["step_api"]["roofline"]["bytes_per_env_step"],
                     "timed K after W warmup + K replay"))
    if "step_api_hipgraph" in v:
        res.append(check("step_api_hipgraph", kn, list(range(W + 3 * K, W + 4 * K)),
                         v["step_api_hipgraph"]["roofline"]["bytes_per_env_step"], "timed graph replay"))
if "step_api_lengths" in v:
    r = v["step_api_lengths"]["roofline"]
    res.append(check("step_api_lengths", r["kernel"], list(range(W + K, W + 2 * K)), r["bytes_per_env_step"],
                     "timed K after W warmup + K replay"))
if "learner_step" in v:
    KL = v["learner_step"]["steps"]
    kn = v["learner_step"]["roofline"]["kernel"].split(" ")[0]
    res.append(check("learner_step", kn, list(range(1 + KL, 1 + 2 * KL)), v["learner_step"]["roofline"]["bytes_per_env_step"],
                     "timed KL after 1 + KL replay"))
os.makedirs(out_dir, exist_ok=True)
with open(os.path.join(out_dir, f"{tag}_step_variants.json"), "w") as fh:
    json.dump({"tag": tag, "bench_line": line, "variants": res}, fh, indent=1)
print(json.dumps(res, indent=1))
