"""Where config 2's step launch spends its time: step_pair_kernel with per-wave timestamps.

Builds (here, no GPU: --build) a variant of ac-solver-caltech_amd/csrc/acx_kernels.hip whose
step_pair_kernel stamps s_memrealtime (the 100 MHz device clock, one time base for the chip) at
its phases and writes them per wave to a buffer passed in acx_step's final_obs argument (the
variant's final_obs write is patched out); the product source is not changed (the stamps are
patched into a copy at text anchors).  On the GPU
box it walks config 2 (65,536 envs, L = 36, Miller-Schupp starts, uniform moves, in place, the
bench's step_api walk) and records a few launches:

    T0 entry, T1 tile converted (its loads arrived), T2 packed + partner planes, T3 moved,
    T4 re-imaged + reset + scalar stores issued, T5 state stores issued, T6 every store done

    python tools/pair_probe.py --build          # -> ab6/libacx_probe.so
    python tools/pair_probe.py [--B 65536] [--K 120] [--at 40,80,119]
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SRC = os.path.join(REPO, "ac-solver-caltech_amd", "csrc", "acx_kernels.hip")
OUT = os.path.join(REPO, "ab6", "libacx_probe.so")
NST = 8  # stamps per wave (7 used)


def patched_source():
    s = open(SRC).read()
    k0 = s.index("__global__ __launch_bounds__(BLOCK, 4) void step_pair_kernel(")
    k1 = s.index("\n}\n", k0) + 2
    body = s[k0:k1]

    def ins(anchor, code, before=True):
        nonlocal body
        assert body.count(anchor) == 1, anchor
        body = body.replace(anchor, code + anchor if before else anchor + code)

    stamp = "__builtin_amdgcn_s_memrealtime()"
    ins("    const int64_t env = r0 + er;\n", f"    uint64_t PT_[{NST}] = {{}};\n    PT_[0] = {stamp};\n", before=False)
    ins("        if (__any(badm != 0u)) {", f"        PT_[1] = {stamp};\n")
    ins("    // the env's move: on a clean env", f"    PT_[2] = {stamp};\n")
    ins("    // this lane's relator re-imaged (a failed env keeps its loaded image)", f"    PT_[3] = {stamp};\n")
    ins("    // the state store.  Relator masks", f"    PT_[4] = {stamp};\n")
    end = (f"{{ PT_[5] = {stamp}; __builtin_amdgcn_s_waitcnt(0); PT_[6] = {stamp}; "
           "if (lane == 0 && a.final_obs) { uint64_t* P_ = reinterpret_cast<uint64_t*>(a.final_obs) + "
           f"((int64_t)blockIdx.x * WPB + wid) * {NST}; for (int i_ = 0; i_ < {NST}; ++i_) P_[i_] = PT_[i_]; }} }}")
    st = body.index("    // the state store.  Relator masks")
    tail = body[st:].replace("return;", "{ " + end + " return; }")
    body = body[:st] + tail[:-2] + "    " + end + "\n}\n"
    anchor = "        if (a.final_obs) {  // final_obs <- the post-move state (rare)"
    assert body.count(anchor) == 1
    body = body.replace(anchor, "        if (false) {  // final_obs carries the probe buffer")
    return s[:k0] + body + s[k1:]


def build():
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    tmp = os.path.join(REPO, "ab6", "acx_kernels_probe.hip")
    with open(tmp, "w") as f:
        f.write(patched_source())
    csrc = os.path.dirname(SRC)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                           "-Wno-pass-failed", "-DACX_ISA_L36_ONLY", "-I" + os.path.join(REPO, "include"), "-I" + csrc,
                           tmp, os.path.join(csrc, "acx_curriculum.hip"), "-o", OUT])
    os.remove(tmp)
    print(OUT)


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * len(v)))]


def run(args):
    import numpy as np
    import torch
    sys.path.insert(0, REPO)
    from bench import ms_starts
    P, I64, I32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32
    lib = ctypes.CDLL(OUT)
    lib.acx_step.argtypes = [P] * 12 + [I64, I32, I32, I32, P]
    dev = torch.device("cuda:0")
    B, L, H = args.B, 36, 200
    start = torch.as_tensor(ms_starts(L, B)).to(dev)
    state = start.clone()
    cnt = torch.zeros(B, dtype=torch.int32, device=dev)
    rew = torch.zeros(B, dtype=torch.int32, device=dev)
    done = torch.zeros(B, dtype=torch.uint8, device=dev)
    trunc = torch.zeros(B, dtype=torch.uint8, device=dev)
    lens = torch.zeros((B, 2), dtype=torch.int32, device=dev)
    err = torch.zeros(B, dtype=torch.uint8, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    acts = torch.randint(0, 12, (args.K, B), dtype=torch.int32, device=dev, generator=g)
    waves = (B + 31) // 32
    at = [int(x) for x in args.at.split(",")]
    bufs = {t: torch.zeros((waves, NST), dtype=torch.int64, device=dev) for t in at}
    s = torch.cuda.current_stream().cuda_stream
    for t in range(args.K):
        pb = bufs[t].data_ptr() if t in bufs else None
        rc = lib.acx_step(state.data_ptr(), state.data_ptr(), acts[t].data_ptr(), start.data_ptr(), cnt.data_ptr(),
                          rew.data_ptr(), done.data_ptr(), trunc.data_ptr(), lens.data_ptr(), pb, err.data_ptr(),
                          None, B, L, H, 1, ctypes.c_void_p(s))
        assert rc == 0
    torch.cuda.synchronize()
    out = {"B": B, "L": L, "waves": waves, "unit": "us (100 MHz device clock)", "launches": {}}
    for t, b in bufs.items():
        T = b.cpu().numpy().astype(np.int64)
        t0 = T[:, 0].min()
        rec = {"kernel_span": float((T[:, 6].max() - t0) / 100.0)}
        names = ["start", "loads_in", "packed", "moved", "imaged_scalars", "stores_issued", "stores_done"]
        for i, n in enumerate(names):
            v = ((T[:, i] - t0) / 100.0).tolist()
            rec["at_" + n] = {q: round(pct(v, p), 3) for q, p in (("p10", .1), ("p50", .5), ("p90", .9), ("max", 1.0))}
        for i in range(1, 7):
            v = ((T[:, i] - T[:, i - 1]) / 100.0).tolist()
            rec[f"d_{names[i - 1]}_to_{names[i]}"] = {q: round(pct(v, p), 3) for q, p in (("p10", .1), ("p50", .5),
                                                                                      ("p90", .9), ("max", 1.0))}
        out["launches"][t] = rec
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--B", type=int, default=65536)
    ap.add_argument("--K", type=int, default=120)
    ap.add_argument("--at", default="40,80,119")
    a = ap.parse_args()
    build() if a.build else run(a)
