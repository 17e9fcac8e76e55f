"""Store pattern variants across buffer placements: allocates 4 resident (T, B, 2L) obs
buffers (B = 2^20, L = 36, T = 200) and times tools/store_pattern.hip feature sets on each,
interleaved, to see which patterns are sensitive to where the buffer lands in HBM
(DESIGN.md "Placement").  usage: store_pattern_alloc.py FLAGS[,FLAGS...]"""
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
lib.sp_tile.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_void_p]
dev = torch.device("cuda:0")
B, T, L = 1 << 20, 200, 36
flags = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [1, 129]
rew = torch.zeros((T, B), dtype=torch.int32, device=dev)
dn = torch.zeros((T, B), dtype=torch.uint8, device=dev)
tr = torch.zeros((T, B), dtype=torch.uint8, device=dev)
act = torch.randint(0, 12, (T, B), dtype=torch.int32, device=dev)
bufs = [torch.zeros((T, B, 2 * L), dtype=torch.int32, device=dev) for _ in range(4)]
s = torch.cuda.current_stream().cuda_stream


def run(obs, f):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    assert lib.sp_tile(obs.data_ptr(), rew.data_ptr(), dn.data_ptr(), tr.data_ptr(), act.data_ptr(), B, T, 2 * L // 4,
                       f, s) == 0
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


for o in bufs:
    for f in flags:
        run(o, f)
res = {f: [[] for _ in bufs] for f in flags}
for rep in range(3):
    for i, o in enumerate(bufs):
        for f in flags:
            res[f][i].append(run(o, f))
print(json.dumps({str(f): [round(min(v), 3) for v in per] for f, per in res.items()}) + "  (ms per buffer)")
