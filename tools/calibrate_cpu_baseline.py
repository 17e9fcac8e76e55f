"""Calibrate bench.py's CPU baseline (oracle/np_port.py, "kind": "port") against the reference
itself: the reference's own ACEnv.step (ac_solver/envs/ac_env.py:91-111, imported from
/root/reference the way tests/golden/make_golden.py does -- build container only) and the port's
PortEnv.step, stepped on the SAME starts (bench.ms_starts: Miller-Schupp, L = 36) with the SAME
uniform actions and the same autoreset on done / truncated, one core, interleaved rounds.

Also checks that the two produce the same states, rewards and done / truncated flags on that
stream (the port is a timing stand-in, so it must do the reference's work).

    python tools/calibrate_cpu_baseline.py [--seconds 10] [--rounds 3] [--out profiles/r04/r04_cpu_calibration.json]

SURVEY §8(d): the port must be within +-20 % of the reference's per-core rate.
"""
import argparse
import json
import os
import platform
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))

from bench import ms_starts  # noqa: E402
from oracle import np_port  # noqa: E402


def run(make_env, starts, actions, horizon, seconds):
    """round-robin over the envs as np_port.run_sample does; returns (env-steps, seconds, trace)"""
    envs = [make_env(s) for s in starts]
    T, B = actions.shape
    steps, t = 0, 0
    trace = []
    t0 = time.perf_counter()
    while True:
        for b in range(B):
            st, r, d, tr, _ = envs[b].step(int(actions[t % T, b]))
            if t < 64:
                trace.append((b, np.array(st).tolist(), float(r), bool(d), bool(tr)))
            if d or tr:
                envs[b].reset()
        steps += B
        t += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            return steps, el, trace


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--L", type=int, default=36)
    ap.add_argument("--horizon", type=int, default=200)
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r04", "r04_cpu_calibration.json"))
    a = ap.parse_args()
    from make_golden import load_reference

    ref = load_reference(a.reference)
    L, H = a.L, a.horizon
    starts = ms_starts(L, 64).astype(np.int64)  # bench.cpu_baseline's rank-0 sample
    actions = np.random.default_rng(0).integers(0, 12, size=(4096, 64))

    def ref_env(s):
        return ref.env.ACEnv(ref.env.ACEnvConfig(initial_state=np.array(s), horizon_length=H))

    def port_env(s):
        return np_port.PortEnv(s, H)

    rates = {"reference": [], "port": []}
    traces = {}
    for _ in range(a.rounds):
        for name, mk in (("reference", ref_env), ("port", port_env)):
            n, el, tr = run(mk, starts, actions, H, a.seconds)
            rates[name].append(n / el)
            traces.setdefault(name, tr)
    same = traces["reference"] == traces["port"]
    ref_rate = float(np.median(rates["reference"]))
    port_rate = float(np.median(rates["port"]))
    res = {
        "what": "one core, 64 envs round-robin, Miller-Schupp starts (bench.ms_starts), uniform actions "
                "(default_rng(0)), L=%d, horizon %d, autoreset on done/truncated; median of %d interleaved rounds of "
                "%.0f s each" % (L, H, a.rounds, a.seconds),
        "reference_ACEnv_step_env_steps_per_s": ref_rate,
        "port_PortEnv_step_env_steps_per_s": port_rate,
        "port_over_reference": port_rate / ref_rate,
        "within_20_percent": abs(port_rate / ref_rate - 1) <= 0.2,
        "rounds": rates,
        "first_64_steps_identical": same,
        "python": platform.python_version(), "numpy": np.__version__,
        "script": "tools/calibrate_cpu_baseline.py",
    }
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "rounds"}, indent=1))


if __name__ == "__main__":
    main()
