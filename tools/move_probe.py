"""Time the packed-code move against the bit-plane prototype (tools/move_probe.hip) on the GPU and
check they agree: 2^20 envs (Miller-Schupp starts, L = 36), T cyclic moves per launch.

    python tools/move_probe.py          (builds tools/libmove_probe.so first if missing)
"""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
SO = os.path.join(HERE, "libmove_probe.so")


def build():
    if not os.path.exists(SO):
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-shared", "-fPIC",
                               "-I", os.path.join(REPO, "include"), "-I", os.path.join(REPO, "ac-solver-caltech_amd", "csrc"),
                               "-I", HERE, os.path.join(HERE, "move_probe.hip"), "-o", SO])
    return SO


def codes_of(starts, L):
    B = starts.shape[0]
    out = np.zeros((B, 8), np.uint32)
    cmap = {1: 0, -1: 1, 2: 2, -2: 3}
    for h in range(2):
        rel = starts[:, h * L:(h + 1) * L]
        n = (rel != 0).sum(1)
        out[:, 6 + h] = n
        code = np.vectorize(lambda v: cmap.get(int(v), 0))(rel).astype(np.uint64)
        for k in range(L):
            out[:, 3 * h + k // 16] |= (code[:, k] << np.uint64(2 * (k % 16))).astype(np.uint32)
    return out


def main():
    import torch  # noqa: F811
    from bench import ms_starts
    lib = ctypes.CDLL(build())
    for f in (lib.probe_codes, lib.probe_planes):
        f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p]
    L, B, T = 36, 1 << 20, 200
    dev = torch.device("cuda:0")
    st0 = torch.as_tensor(codes_of(ms_starts(L, 1190), L).view(np.int32)).to(dev)[torch.arange(B, device=dev) % 1190]
    acts = torch.randint(0, 2**31 - 1, (T,), dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    res = {}
    outs = {}
    for name, f in (("codes", lib.probe_codes), ("planes", lib.probe_planes)):
        ms = []
        for rep in range(4):
            st = st0.clone().contiguous()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            assert f(st.data_ptr(), acts.data_ptr(), T, L, B, s) == 0
            e1.record()
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
        outs[name] = st
        res[name] = {"ms": [round(x, 4) for x in ms], "us_per_2^20_env_step": round(min(ms[1:]) / T * 1e3, 3)}
    res["equal"] = bool(torch.equal(outs["codes"], outs["planes"]))
    res["T"], res["B"], res["L"] = T, B, L
    print(json.dumps(res))


if __name__ == "__main__":
    main()
