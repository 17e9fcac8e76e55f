"""Partial-line read calibration (tools/line_probe.hip): how many HBM bytes a read of part of a
128-B line moves, by time against the whole-line read of the same lines, and what rocprofv3's
read counters say for it (run this under `rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum
TCC_BUBBLE_sum` for the counters).  A 2 GiB buffer (past the 256 MiB Infinity Cache), each kind
REPS times interleaved.

    python tools/line_probe.py [--reps 5]     (builds tools/libline_probe.so on first use)
"""
import argparse
import ctypes
import json
import os
import statistics
import subprocess

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libline_probe.so")
KINDS = {0: ("whole line", 128), 1: ("first 64-B sector", 64), 2: ("second 64-B sector", 64),
         3: ("one 16-B chunk", 16), 4: ("32 B across the sector boundary", 32)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    if not os.path.exists(SO):
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                               os.path.join(HERE, "line_probe.hip"), "-o", SO])
    lib = ctypes.CDLL(SO)
    lib.line_probe_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]
    dev = torch.device("cuda:0")
    lines = (2 << 30) // 128
    buf = torch.randint(-2, 3, (lines * 32,), dtype=torch.int32, device=dev)
    out = torch.zeros(256 * 8, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    ms = {k: [] for k in KINDS}
    for rep in range(a.reps + 1):
        for k in KINDS:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            assert lib.line_probe_run(k, buf.data_ptr(), lines, out.data_ptr(), s) == 0
            e1.record()
            torch.cuda.synchronize()
            if rep:
                ms[k].append(e0.elapsed_time(e1))
    res = {"lines": lines, "buffer_bytes": lines * 128}
    full = statistics.median(ms[0])
    for k, (what, req) in KINDS.items():
        m = statistics.median(ms[k])
        res[what] = {"ms": round(m, 4), "requested_bytes_per_line": req,
                     "requested_GBs": round(lines * req / m / 1e6, 1),
                     "whole_line_equivalent_GBs": round(lines * 128 / m / 1e6, 1),
                     "time_vs_whole_line": round(m / full, 3)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
