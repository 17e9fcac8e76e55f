"""The per-call step API against the copy ceiling of its traffic, in one process and allocation:
acx_step (B envs, state in place, every output) vs a float4 grid-stride copy and a tile-shaped
copy of the same state bytes (tools/store_pattern.hip) and torch copy_.

    python tools/step_probe.py [L ...]      (default 36 128)"""
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ac-solver-caltech_amd"))
sys.path.insert(0, REPO)
from acx import ops  # noqa: E402
from bench import ms_starts  # noqa: E402

sp = ctypes.CDLL(os.path.join(REPO, "tools", "libstore_pattern.so"))
sp.sp_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int64, ctypes.c_int,
                       ctypes.c_void_p]
dev = torch.device("cuda:0")
B, H, K = 1 << 20, 200, 50
out = {}


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    return best


for L in [int(x) for x in sys.argv[1:]] or [36, 128]:
    starts = torch.as_tensor(ms_starts(L, B)).to(dev)
    st = starts.clone()
    cnt = torch.zeros(B, dtype=torch.int32, device=dev)
    rew = torch.empty(B, dtype=torch.int32, device=dev)
    dn = torch.empty(B, dtype=torch.uint8, device=dev)
    tr = torch.empty(B, dtype=torch.uint8, device=dev)
    lens = torch.empty((B, 2), dtype=torch.int32, device=dev)
    err = torch.empty(B, dtype=torch.uint8, device=dev)
    acts = torch.randint(0, 12, (K, B), dtype=torch.int32, device=dev)

    def steps():
        for t in range(K):
            ops.step(st, acts[t], state_out=st, reset_state=starts, step_count=cnt, horizon=H, cyclical=True,
                     reward=rew, done=dn, truncated=tr, lengths=lens, err=err)

    ms = timed(steps) / K
    sb = 16 * L + 27
    dst = torch.empty_like(st)
    n16 = B * 2 * L // 4
    s = torch.cuda.current_stream().cuda_stream
    c0 = timed(lambda: sp.sp_copy(st.data_ptr(), dst.data_ptr(), n16, 0, B, 2 * L // 4, s))
    c1 = timed(lambda: sp.sp_copy(st.data_ptr(), dst.data_ptr(), n16, 1, B, 2 * L // 4, s))
    ct = timed(lambda: dst.copy_(st))
    cb = 2 * B * 8 * L
    out[f"L{L}"] = {"step_ms": ms, "step_TBps": B * sb / ms / 1e9, "step_frac": B * sb / ms / 1e9 / 8,
                    "copy16_TBps": cb / c0 / 1e9, "tile_copy_TBps": cb / c1 / 1e9, "torch_copy_TBps": cb / ct / 1e9}
    del starts, st, dst, acts
    torch.cuda.empty_cache()
print(json.dumps(out))
