"""Rollout speed vs how the (T, B, 2L) obs buffer is allocated.  In each of N fresh processes:
the obs buffer from torch's caching allocator, from hipExtMallocWithFlags(hipDeviceMallocContiguous)
(physically contiguous), and from plain hipMalloc; the same 200-step rollout (2^20 envs, L = 36)
timed into each (best of 3).  Prints one JSON line per process.

    python tools/alloc_probe4.py [N]
"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import ctypes, json, sys, torch
sys.path.insert(0, %(pkg)r); sys.path.insert(0, %(repo)r)
from bench import ms_starts
from acx import _lib
lib = _lib.load()
hip = ctypes.CDLL("libamdhip64.so")
dev = torch.device("cuda:0")
L, B, T, H = 36, 1 << 20, 200, 200
nbytes = T * B * 2 * L * 4
starts = torch.as_tensor(ms_starts(L, B)).to(dev)
g = torch.Generator(device=dev); g.manual_seed(0)
acts = torch.randint(0, 12, (T, B), dtype=torch.int32, device=dev, generator=g)
packed = torch.empty(((T + 7) // 8, B), dtype=torch.int32, device=dev)
rew = torch.zeros((T, B), dtype=torch.int32, device=dev)
dn = torch.zeros((T, B), dtype=torch.uint8, device=dev)
tr = torch.zeros((T, B), dtype=torch.uint8, device=dev)
err = torch.zeros(B, dtype=torch.uint8, device=dev)
ec = torch.zeros(1, dtype=torch.int32, device=dev)
stream = torch.cuda.current_stream(dev).cuda_stream
def roll(obs_ptr):
    state = starts.clone(); cnt = torch.zeros(B, dtype=torch.int32, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); e0.record()
    lib.acx_pack_actions(acts.data_ptr(), packed.data_ptr(), T, B, stream)
    st = lib.acx_rollout_packed(state.data_ptr(), packed.data_ptr(), starts.data_ptr(), cnt.data_ptr(), obs_ptr,
                                rew.data_ptr(), dn.data_ptr(), tr.data_ptr(), err.data_ptr(), ec.data_ptr(),
                                T, B, L, H, 1, stream)
    e1.record(); torch.cuda.synchronize()
    assert st == 0
    return e0.elapsed_time(e1)
def best(ptr):
    roll(ptr)
    return round(min(roll(ptr) for _ in range(3)), 3)
out = {}
def torch_alloc():
    obs = torch.zeros((T, B, 2 * L), dtype=torch.int32, device=dev)
    out["torch"] = best(obs.data_ptr())
    del obs; torch.cuda.empty_cache()
order = sys.argv[1] if len(sys.argv) > 1 else "torch-first"
out["order"] = order
if order == "torch-first":
    torch_alloc()
for name, flag in (("contiguous", 4), ("hipMalloc", None)):
    p = ctypes.c_void_p()
    if flag is None:
        rc = hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(nbytes))
    else:
        rc = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(nbytes), ctypes.c_uint(flag))
    if rc != 0:
        out[name] = f"alloc failed rc={rc}"
        continue
    hip.hipMemset(p, 0, ctypes.c_size_t(nbytes)); torch.cuda.synchronize()
    out[name] = best(p.value)
    hip.hipFree(p)
if order != "torch-first":
    torch_alloc()
print(json.dumps(out))
'''

if __name__ == "__main__":
    code = CHILD % {"pkg": os.path.join(REPO, "ac-solver-caltech_amd"), "repo": REPO}
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    for i in range(n):
        order = "torch-first" if i % 2 == 0 else "torch-last"
        r = subprocess.run([sys.executable, "-c", code, order], capture_output=True, text=True, timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        print(line[-1] if line else json.dumps({"error": r.stderr[-600:]}), flush=True)
