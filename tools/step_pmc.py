"""A short program for rocprofv3 --pmc passes over the two in-place step kernels: acx_step
(step_kernel) and acx_step_lengths (step_lengths_kernel) on the same walk -- 2^20 envs,
Miller-Schupp starts, uniform moves, horizon 200 -- W + K calls each, at L = 128 then L = 36.

    rocprofv3 --pmc SQ_WAVE_CYCLES ... -d gpurun_out/pmc -o pmc -- python3 tools/step_pmc.py
    ... -- python3 tools/step_pmc.py --L 36 --B 65536 --K 50   (config 2's launch: step_pair_kernel)
"""
import argparse
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "ac-solver-caltech_amd"))
from bench import ms_starts  # noqa: E402
from acx import ops  # noqa: E402


def run(L, B=1 << 20, W=2, K=5, H=200):
    dev = torch.device("cuda:0")
    starts = torch.as_tensor(ms_starts(L, B)).to(dev)
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    acts = torch.randint(0, 12, (W + K, B), dtype=torch.int32, device=dev, generator=g)
    for lengths_in in (False, True):
        st = starts.clone()
        cnt = torch.zeros(B, dtype=torch.int32, device=dev)
        lens = torch.full((B, 2), L, dtype=torch.int32, device=dev)
        for t in range(W + K):
            ops.step(st, acts[t], state_out=st, reset_state=starts, step_count=cnt, horizon=H, cyclical=True,
                     lengths=lens, lengths_in=lengths_in)
        torch.cuda.synchronize()


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=0, help="one L only (default: 128 then 36)")
    ap.add_argument("--B", type=int, default=1 << 20)
    ap.add_argument("--K", type=int, default=5)
    a = ap.parse_args()
    for L in ((a.L,) if a.L else (128, 36)):
        run(L, B=a.B, K=a.K)
    print("ok")
