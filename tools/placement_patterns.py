"""Which store patterns are placement-sensitive?  For several fresh (T, B, 2L) int32 buffers
(T = 20, B = 2^20, L = 36: the driver's obs trajectory), time on each buffer: the rollout's bare
obs store pattern (tools/store_pattern.hip tile_pattern<NT>: every wave streams its 64-row tile,
18 KB, per step) at 8 / 6 / 4 / 2 resident waves per SIMD (extra dynamic LDS caps the blocks
per CU), and a linear grid-stride fill.  One JSON line per buffer on stderr, a summary on stdout.

    python tools/placement_patterns.py [trials]"""
import ctypes
import json
import os
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
so = os.path.join(HERE, "libstore_pattern.so")
if not os.path.exists(so):
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", "-o", so,
                           os.path.join(HERE, "store_pattern.hip")])
lib = ctypes.CDLL(so)
lib.sp_tile_occ.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
lib.sp_linear.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
trials = int(sys.argv[1]) if len(sys.argv) > 1 else 6
dev = torch.device("cuda:0")
B, T, L = 1 << 20, 20, 36
rc = 2 * L // 4
s = torch.cuda.current_stream().cuda_stream
# static LDS of tile_pattern: 4 x 64 x 18 dwords = 18 KB per block; 160 KB per CU
PADS = {8: 0, 6: 9 * 1024, 4: 22 * 1024, 2: 62 * 1024}
nbytes = T * B * 2 * L * 4


def best_ms(fn, reps=4):
    fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1))
    return min(out)


rows = []
keep = []
for trial in range(trials):
    obs = torch.empty((T, B, 2 * L), dtype=torch.int32, device=dev)
    obs.zero_()
    r = {"trial": trial}
    for w, pad in PADS.items():
        ms = best_ms(lambda: lib.sp_tile_occ(obs.data_ptr(), B, T, rc, pad, s))
        r[f"tile_w{w}_TBps"] = round(nbytes / ms / 1e9, 3)
    ms = best_ms(lambda: lib.sp_linear(obs.data_ptr(), nbytes // 16, 8192, s))
    r["linear_TBps"] = round(nbytes / ms / 1e9, 3)
    rows.append(r)
    print(json.dumps(r), file=sys.stderr, flush=True)
    keep.append(obs)  # a new region every trial
print(json.dumps({"B": B, "T": T, "L": L, "rows": rows}))
