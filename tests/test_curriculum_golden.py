"""The PPO start-state curriculum against the reference's own training loop
(tests/golden/curriculum.npz, made by tests/golden/make_curriculum_golden.py, which runs
ac_solver/agents/training.py:ppo_training_loop itself with recorded moves).

CPU: oracle/curriculum.py (the env side of training.py:221-352 over the oracle env step) with
acx.agents.CurriculumRecord (the host bookkeeping: success_record, ACMoves_hist, the seeded
round-2 draws) reproduce every step -- rewards, done, truncated, curr_states after the loop's
processing, every env's state -- and the final records.  The GPU twin is
tests/test_gpu_learner.py::test_learner_env_matches_reference_training_loop."""
import json
import os
import random

import numpy as np
import pytest

from oracle import curriculum as C

HERE = os.path.dirname(os.path.abspath(__file__))


def golden_cases():
    with open(os.path.join(HERE, "golden", "curriculum.json")) as f:
        meta = json.load(f)
    z = np.load(os.path.join(HERE, "golden", "curriculum.npz"))
    return [(name, m, {k.split("__", 1)[1]: z[k] for k in z.files if k.startswith(name + "__")})
            for name, m in meta.items()]


def check_final(rec, m):
    assert sorted(rec.success_record["solved"]) == m["solved"]
    assert sorted(rec.success_record["unsolved"]) == m["unsolved"]
    assert sorted(rec.states_processed) == m["states_processed"]
    assert {str(k): [int(a) for a in v] for k, v in rec.ACMoves_hist.items()} == m["ACMoves_hist"]


@pytest.mark.parametrize("case", golden_cases(), ids=lambda c: c[0])
def test_oracle_and_host_record_match_reference_training_loop(case):
    from acx.agents import CurriculumRecord
    name, m, g = case
    init = g["initial_states"].astype(np.int32)
    B, T, U = m["num_envs"], m["num_steps"], m["updates"]
    env = C.RolloutEnvs(init, B, m["horizon"])
    rng = random.Random()
    rec = CurriculumRecord(len(init), B, m["repeat_solved_prob"], rng=rng)
    rec.curr_states, rec.states_processed = env.curr_states, env.states_processed  # one set of books
    n_host = 0
    for u in range(1, U + 1):
        rng.seed(m["seed"] + u)  # training.py:204
        for s in range(T):
            t = (u - 1) * T + s
            res = env.step(g["actions"][t].astype(np.int64), lambda i: rec.draw(), on_done=rec.on_done)
            assert np.array_equal(res["reward"], g["reward"][t]), (name, t)
            assert np.array_equal(res["done"].astype(np.uint8), g["done"][t]), (name, t)
            assert np.array_equal(res["truncated"].astype(np.uint8), g["truncated"][t]), (name, t)
            assert env.curr_states == list(g["curr_states"][t]), (name, t)
            assert np.array_equal(env.state, g["post_state"][t].astype(np.int32)), (name, t)
            n_host += int(res["picked_by_host"].sum())
    check_final(rec, m)
    assert n_host > 10 and len(m["solved"]) > 0  # the golden exercises round 2 and solved episodes
