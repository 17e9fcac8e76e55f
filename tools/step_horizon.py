"""Config 5's kernel launch by launch: the bench's random-action walk at L = 128, 2^20 envs,
horizon 200 (Miller-Schupp starts, seed 0, in place, same-step autoreset) through
acx_step_lengths, every launch timed with its own HIP events, and beside each its bytes:
  live    -- ceil(n/4) x 16 B read per relator, a changed relator's chunks inside its old or new
             letters written, + 43 B of lengths and scalars (bench.py's accounting);
  sectors -- the same with each relator's reads rounded up to the 64-B sectors HBM moves.
So the time per launch can be read against what it must move as the relators grow through the
horizon and drop at the synchronised reset.  The byte accounting is an untimed replay of the
same steps from a snapshot (the kernel is deterministic).

    python tools/step_horizon.py [--steps 210] [--L 128]
"""
import argparse
import json
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "ac-solver-caltech_amd"))
from bench import ms_starts  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=210)
    ap.add_argument("--L", type=int, default=128)
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--ceiling-at", type=int, default=0,
                    help="after the timed walk, replay to this step and run the bare live-chunk read "
                         "shape (tools/stream_ceiling.hip live_tile) on that state and its lengths")
    a = ap.parse_args()
    from acx import ops

    L, B, K, H = a.L, a.batch, a.steps, 200
    dev = torch.device("cuda:0")
    starts = torch.as_tensor(ms_starts(L, B)).to(dev)
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    acts = torch.randint(0, 12, (K, B), dtype=torch.int32, device=dev, generator=g)
    st = starts.clone()
    cnt = torch.zeros(B, dtype=torch.int32, device=dev)
    lens = torch.full((B, 2), L, dtype=torch.int32, device=dev)
    rew = torch.empty(B, dtype=torch.int32, device=dev)
    dn = torch.empty(B, dtype=torch.uint8, device=dev)
    tr = torch.empty(B, dtype=torch.uint8, device=dev)
    err = torch.zeros(B, dtype=torch.uint8, device=dev)
    ec = torch.zeros(1, dtype=torch.int32, device=dev)

    def step(x):
        ops.step(st, x, state_out=st, reset_state=starts, step_count=cnt, horizon=H, cyclical=True, reward=rew,
                 done=dn, truncated=tr, lengths=lens, err=err, err_count=ec, lengths_in=True)

    step(acts[0])  # (L, L) on entry: the first call reads whole rows; from here lengths are exact
    snap = (st.clone(), cnt.clone(), lens.clone())
    live, sect = [], []
    for t in range(1, K):
        before, nb = st.clone(), lens.clone()
        step(acts[t])
        ch = (before.view(B, 2, L) != st.view(B, 2, L)).any(2)
        c_old = (nb.clamp(0, L) + 3) // 4
        c_new = (lens.clamp(0, L) + 3) // 4
        wr = float((torch.maximum(c_old, c_new) * ch).sum().item()) * 16
        live.append(float(c_old.sum().item()) * 16 + wr + 43 * B)
        sect.append(float(((nb.clamp(0, L) + 15) // 16).sum().item()) * 64 + wr + 43 * B)
        del before, nb
    for x, y in zip((st, cnt, lens), snap):
        x.copy_(y)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(1, K)]
    for t in range(1, K):
        ev[t - 1][0].record()
        step(acts[t])
        ev[t - 1][1].record()
    torch.cuda.synchronize()
    ms = [e0.elapsed_time(e1) for e0, e1 in ev]
    rows = [{"step": t, "ms": round(m, 4), "live_MB": round(lb / 1e6, 1), "sector_MB": round(sb / 1e6, 1),
             "live_TBps": round(lb / m / 1e9, 3), "sector_TBps": round(sb / m / 1e9, 3)}
            for t, m, lb, sb in zip(range(1, K), ms, live, sect)]
    tot_ms = sum(ms)
    ceil = None
    if a.ceiling_at:
        import ctypes
        import subprocess
        so = os.path.join(REPO, "tools", "libstream_ceiling.so")
        src = os.path.join(REPO, "tools", "stream_ceiling.hip")
        if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
            subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-shared",
                                   "-fPIC", src, "-o", so])
        cl = ctypes.CDLL(so)
        cl.probe_live.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                                  ctypes.c_void_p, ctypes.c_void_p]
        for x, y in zip((st, cnt, lens), snap):
            x.copy_(y)
        for t in range(1, a.ceiling_at):
            step(acts[t])
        lb = float(((lens.clamp(0, L) + 3) // 4).sum().item()) * 16
        sbytes = float(((lens.clamp(0, L) + 15) // 16).sum().item()) * 64
        scratch = st.clone()
        outb = torch.zeros(1 << 16, dtype=torch.int32, device=dev)
        ceil = {"at_step": a.ceiling_at, "live_read_MB": round(lb / 1e6, 1), "sector_read_MB": round(sbytes / 1e6, 1)}
        for wr in (0, 1, 2):
            for lds, occ in ((40 * 1024, 4), (20 * 1024, 8)):
                ts = []
                for r in range(6):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    assert cl.probe_live(wr, scratch.data_ptr(), lens.data_ptr(), B, lds, outb.data_ptr(),
                                         torch.cuda.current_stream().cuda_stream) == 0
                    e1.record()
                    torch.cuda.synchronize()
                    if r:
                        ts.append(e0.elapsed_time(e1))
                m = statistics.median(ts)
                ceil[f"{('read', 'rw', 'rw_sectors')[wr]}_occ{occ}"] = {"ms": round(m, 4), "live_read_TBps": round(lb / m / 1e9, 3),
                                                             "sector_read_TBps": round(sbytes / m / 1e9, 3)}
        del scratch
    out = {"what": "tools/step_horizon.py: acx_step_lengths launch by launch on the bench's config-5 walk "
                   f"(L={L}, B={B}, horizon {H}, steps 1..{K - 1}; step 0 read whole rows)",
           "total_ms": round(tot_ms, 3), "live_TBps_overall": round(sum(live) / tot_ms / 1e9, 3),
           "sector_TBps_overall": round(sum(sect) / tot_ms / 1e9, 3),
           "median_ms": round(statistics.median(ms), 4), "err_count": int(ec.item()), "ceiling": ceil,
           "launches": rows}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
