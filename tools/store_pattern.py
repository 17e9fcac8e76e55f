"""Run tools/store_pattern.hip (built here with hipcc --offload-arch=gfx950 -O3 -shared -fPIC,
or on first use).  Prints achieved GB/s (all bytes moved: obs + scalars + actions) per feature
combination of the rollout access pattern at B = 2^20, L = 36, T = 200."""
import ctypes, json, os, subprocess, sys
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
so = os.path.join(HERE, "libstore_pattern.so")
if not os.path.exists(so):
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", "-o", so,
                           os.path.join(HERE, "store_pattern.hip")])
lib = ctypes.CDLL(so)
lib.sp_tile.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_void_p]
lib.sp_linear.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
lib.sp_chunk.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
dev = torch.device("cuda:0")
B, T, L = int(os.environ.get("SP_B", 1 << 20)), int(os.environ.get("SP_T", 200)), 36
rc = 2 * L // 4
obs = torch.zeros((T, B, 2 * L), dtype=torch.int32, device=dev)
rew = torch.zeros((T, B), dtype=torch.int32, device=dev)
dn = torch.zeros((T, B), dtype=torch.uint8, device=dev)
tr = torch.zeros((T, B), dtype=torch.uint8, device=dev)
act = torch.randint(0, 12, (T, B), dtype=torch.int32, device=dev)
obs_bytes = obs.numel() * 4
s = torch.cuda.current_stream().cuda_stream
res = {}


def timeit(fn, name, nbytes):
    assert fn() == 0
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); e1.record(); torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    res[name] = {"ms": round(best, 4), "GBps": round(nbytes / best / 1e6, 1)}


NAMES = {1: "NT", 2: "SCAL", 4: "ACT8", 8: "ACTPF", 16: "LDS", 32: "ACT32", 64: "PACK8", 128: "BLK", 256: "ROT"}
import sys as _sys
flag_list = [int(x) for x in _sys.argv[1].split(",")] if len(_sys.argv) > 1 else [1, 5, 33, 65, 19, 23, 51, 83, 1, 19]
for flags in flag_list:
    nb = obs_bytes + (T * B * 6 if flags & 2 else 0) + (T * B * 4 if flags & 44 else 0) + (T * B // 2 if flags & 64 else 0)
    name = "tile_" + ("+".join(v for k, v in NAMES.items() if flags & k) or "plain")
    name = name if name not in res else name + "_again"
    timeit(lambda: lib.sp_tile(obs.data_ptr(), rew.data_ptr(), dn.data_ptr(), tr.data_ptr(), act.data_ptr(), B, T, rc,
                               flags, s), name, nb)
lib.sp_tile2.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
if os.environ.get("SP_TILE2"):
    timeit(lambda: lib.sp_tile2(obs.data_ptr(), B, T, rc, s), "tile2_NT", obs_bytes)
for blocks in [int(x) for x in os.environ.get("SP_BLOCKS", "8192").split(",")]:
    timeit(lambda: lib.sp_linear(obs.data_ptr(), obs_bytes // 16, blocks, s), f"linear_{blocks}", obs_bytes)
for per in [int(x) for x in os.environ.get("SP_PER", "").split(",") if x]:
    timeit(lambda: lib.sp_chunk(obs.data_ptr(), obs_bytes // 16, per, s), f"chunk_{per}", obs_bytes)
timeit(lambda: (obs.fill_(3), 0)[1], "torch_fill", obs_bytes)
print(json.dumps(res, indent=0))
