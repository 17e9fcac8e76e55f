#!/bin/bash
# Which box class is this (tools/README: the K = 20 headline lands at 1.10 ms on some boxes and
# 1.34-1.38 ms on most)?  The box's HBM vendor / VBIOS / clocks beside the headline launch alone
# (no CPU baseline, no variants), appended to gpurun_out/box_rate.jsonl.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
V=$(rocm-smi --showmemvendor 2>/dev/null | grep -o "memory vendor: [A-Za-z]*" | head -1 | sed 's/memory vendor: //')
B=$(rocm-smi --showvbios 2>/dev/null | grep -o "VBIOS version: [^ ]*" | head -1 | sed 's/VBIOS version: //')
H=$(hostname 2>/dev/null | md5sum | cut -c1-8)
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-step-api --no-learner --no-graph --no-bfs \
  --no-search --no-desync --no-obs8 --no-config2 > gpurun_out/box_rate_bench.json 2> gpurun_out/box_rate_bench.err || exit 1
python - "$V" "$B" "$H" <<'PY' >> gpurun_out/box_rate.jsonl
import json, sys
d = json.loads([l for l in open("gpurun_out/box_rate_bench.json") if l.strip().startswith("{")][-1])
print(json.dumps({"hbm_vendor": sys.argv[1], "vbios": sys.argv[2], "host": sys.argv[3], "value": d["value"],
                  "kernel_ms": d["roofline"]["kernel_ms"], "frac": d["roofline"]["frac"]}))
PY
tail -1 gpurun_out/box_rate.jsonl
