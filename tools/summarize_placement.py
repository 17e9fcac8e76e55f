"""Summarise tools/profile_placement.sh: per pass, the counters of the last four rollout_kernel
dispatches (slow, slow, fast, fast, as tools/placement_pmc.py launches them) with that pass's
own classification and launch times.

    python tools/summarize_placement.py gpurun_out/prof_place_TAG [out.json]
"""
import csv
import json
import os
import sys
from collections import defaultdict


def main(d, out=None):
    res = {}
    for pas in sorted(os.listdir(d)):
        f = os.path.join(d, pas, "r_counter_collection.csv")
        if not os.path.exists(f):
            continue
        log = open(os.path.join(d, pas + ".log")).read().splitlines()
        cls = next((json.loads(x) for x in log if x.startswith('{"classify_ms"')), None)
        disp = defaultdict(dict)
        for row in csv.DictReader(open(f)):
            if "rollout_kernel" not in row["Kernel_Name"]:
                continue
            k = int(row["Dispatch_Id"])
            disp[k][row["Counter_Name"]] = disp[k].get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
            disp[k]["_ns"] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
        last = sorted(disp)[-4:]
        res[pas] = {"classify": cls, "dispatches": [{"kind": cls["order"][i] if cls else "?", "ms": disp[k]["_ns"] / 1e6,
                                                     **{c: v for c, v in sorted(disp[k].items()) if c != "_ns"}}
                                                    for i, k in enumerate(last)]}
    js = json.dumps(res, indent=1)
    if out:
        open(out, "w").write(js)
    return res


if __name__ == "__main__":
    r = main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
    for pas, v in r.items():
        print(pas, v["classify"]["classify_ms"] if v["classify"] else None)
        for dd in v["dispatches"]:
            vals = [(c, x) for c, x in dd.items() if c not in ("kind", "ms")]
            print("  ", dd["kind"], round(dd["ms"], 3), " ".join(f"{c.replace('ACX_', '')}={x:.3g}" for c, x in vals))
