"""Run tools/store_pattern.hip (build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC)."""
import ctypes, json, os, subprocess, sys
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
so = os.path.join(HERE, "libstore_pattern.so")
if not os.path.exists(so):
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", "-o", so,
                           os.path.join(HERE, "store_pattern.hip")])
lib = ctypes.CDLL(so)
lib.sp_tile.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
lib.sp_linear.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
dev = torch.device("cuda:0")
B, T, L = 1 << 20, 200, 36
rc = 2 * L // 4
obs = torch.zeros((T, B, 2 * L), dtype=torch.int32, device=dev)
nbytes = obs.numel() * 4
s = torch.cuda.current_stream().cuda_stream
res = {}
def timeit(fn, name):
    fn(); torch.cuda.synchronize()
    best = 1e9
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); e1.record(); torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    res[name] = {"ms": best, "GBps": nbytes / best / 1e6}
timeit(lambda: lib.sp_tile(obs.data_ptr(), B, T, rc, 0, s), "tile_pattern")
timeit(lambda: lib.sp_tile(obs.data_ptr(), B, T, rc, 1, s), "tile_pattern_nt")
for blocks in (2048, 8192, 65536):
    timeit(lambda: lib.sp_linear(obs.data_ptr(), nbytes // 16, blocks, s), f"linear_{blocks}")
timeit(lambda: obs.fill_(3), "torch_fill")
print(json.dumps(res))
