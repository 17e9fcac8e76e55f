"""Which of acx_step_learner's outputs cost what?  B = 2^20, L = 36 and 128: times 50 calls with
subsets of the learner-side outputs (float32 obs, episode move history, the rest) and reports
each subset's algorithmic bytes per env-step and fraction of 8 TB/s -- the float32 obs (8L B, the
state's second store) measured separately from the int32 state store.

    python tools/learner_ablation.py [L ...]"""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ac-solver-caltech_amd"))
sys.path.insert(0, REPO)
from bench import ms_starts  # noqa: E402
from acx import _lib  # noqa: E402

lib = _lib.load()
dev = torch.device("cuda:0")
B, K, H, HC = 1 << 20, 50, 200, 200
stream = torch.cuda.current_stream().cuda_stream
p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
out = {}
for L in [int(x) for x in sys.argv[1:]] or [36, 128]:
    starts = torch.as_tensor(ms_starts(L, B)).to(dev)
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    acts = torch.randint(0, 12, (K, B), dtype=torch.int64, device=dev, generator=g)
    obs = torch.zeros((B, 2 * L), dtype=torch.float32, device=dev)
    rf = torch.zeros(B, dtype=torch.float32, device=dev)
    df = torch.zeros(B, dtype=torch.float32, device=dev)
    dn = torch.zeros(B, dtype=torch.uint8, device=dev)
    tr = torch.zeros(B, dtype=torch.uint8, device=dev)
    hist = torch.zeros((HC, B), dtype=torch.uint8, device=dev)
    eplen = torch.zeros(B, dtype=torch.int32, device=dev)
    err = torch.zeros(B, dtype=torch.uint8, device=dev)

    def run(use_obs, use_hist, use_rest):
        st = starts.clone()
        cnt = torch.zeros(B, dtype=torch.int32, device=dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for t in range(K):
            rc = lib.acx_step_learner(st.data_ptr(), None, acts[t].data_ptr(), starts.data_ptr(), cnt.data_ptr(),
                                      p(obs if use_obs else None), p(rf if use_rest else None),
                                      p(df if use_rest else None), p(dn), p(tr), p(hist if use_hist else None),
                                      HC if use_hist else 0, p(eplen if use_rest else None), None, p(err), None, B, L,
                                      H, 1, stream)
            assert rc == 0
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / K

    # bytes per env-step: state in/out 16L, int64 action 8, count in/out 8, done/trunc 2, err 1;
    # + float32 obs 8L; + episode history 1; + reward/done f32 and episode length 12
    base = 16 * L + 19
    cases = {"all": ((1, 1, 1), base + 8 * L + 13), "no_hist": ((1, 0, 1), base + 8 * L + 12),
             "no_obs": ((0, 1, 1), base + 13), "no_obs_no_hist": ((0, 0, 1), base + 12), "bare": ((0, 0, 0), base)}
    res = {k: [] for k in cases}
    for rep in range(3):
        for k, (c, _) in cases.items():
            res[k].append(run(*c))
    out[f"L{L}"] = {k: {"us_per_step": round(min(v) * 1e3, 1), "bytes_per_env_step": cases[k][1],
                        "frac": round(B * cases[k][1] / (min(v) / 1e3) / 8e12, 3)} for k, v in res.items()}
    out[f"L{L}"]["obs_f32_store_us"] = round((min(res["all"]) - min(res["no_obs"])) * 1e3, 1)
    del starts, acts, obs, hist
print(json.dumps(out))
