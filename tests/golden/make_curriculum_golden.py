"""Generate tests/golden/curriculum.npz + curriculum.json: the reference's own PPO rollout phase
(ac_solver/agents/training.py:138-356, `ppo_training_loop`) driven for a few updates, with its
start-state curriculum recorded step by step.

    python tests/golden/make_curriculum_golden.py [--reference /root/reference]

What runs is the reference function itself, imported from /root/reference (as make_golden.py
does for the env and the searches).  What stands in around it:
  * gymnasium is not installed: `RecVecEnv` restates gymnasium 0.28.1
    SyncVectorEnv's same-step autoreset (reset() without options on done | truncated, the
    final step's info under infos["final_info"][i] with the "_final_info" mask) around the
    reference's ACEnv objects -- that part stays parity unpinned, as DESIGN.md says;
  * the policy is `ScriptedAgent`: uniform random moves from a seeded generator, skipping moves
    that would raise in ACMove (an emptied relator), so the loop never aborts; its logprob /
    value heads are two tiny parameters so the PPO update after each rollout runs as written;
  * wandb is a stub (wandb_log=False); the loop's out/ and experiments/ files go to a temp dir.

Recorded per env step t: the moves taken, reward / done / truncated as envs.step returned them,
`curr_states` after the loop processed step t (the curriculum's assignment), and every env's
state after step t (post autoreset and post curriculum reset); at the end success_record,
ACMoves_hist and states_processed.  The seeds are the reference's own: random / np.random /
torch seeded with args.seed + update at the start of each update (training.py:203-206).
"""
from __future__ import annotations

import argparse
import copy
import importlib
import json
import os
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import load_reference  # noqa: E402


def load_training(root):
    ref = load_reference(root)
    import torch  # noqa: F401  (the reference module imports it)
    wandb = types.ModuleType("wandb")
    wandb.init = lambda *a, **k: None
    wandb.log = lambda *a, **k: None
    sys.modules["wandb"] = wandb
    m = types.ModuleType("ac_solver.agents")
    m.__path__ = [os.path.join(root, "ac_solver", "agents")]
    sys.modules["ac_solver.agents"] = m
    ref.training = importlib.import_module("ac_solver.agents.training")
    return ref


class RecEnv:
    """One env of the vector: the reference ACEnv, with the training loop's curriculum resets
    (`envs.envs[i].reset(options=...)`, training.py:352) passed through."""

    def __init__(self, inner):
        self.inner = inner

    @property
    def unwrapped(self):
        return self.inner

    def reset(self, *, seed=None, options=None):
        return self.inner.reset(seed=seed, options=options)


class RecVecEnv:
    """gymnasium 0.28.1 SyncVectorEnv semantics (same-step autoreset) over reference ACEnvs."""

    def __init__(self, ref, initial_states, num_envs, horizon):
        self.ref = ref
        L = initial_states[0].shape[0] // 2
        self.envs = []
        for i in range(num_envs):
            cfg = ref.env.ACEnvConfig.from_dict({"initial_state": initial_states[i], "horizon_length": horizon,
                                                 "use_supermoves": False})
            self.envs.append(RecEnv(ref.env.ACEnv(cfg)))
        self.num_envs = num_envs
        self.single_observation_space = types.SimpleNamespace(shape=(2 * L,))
        self.single_action_space = types.SimpleNamespace(shape=())
        self.steps = []  # per envs.step call: actions, reward, done, truncated
        self.post_states = []  # env states when the next step starts (= after the loop's processing)
        self.curr_snap = []
        self.curr_states = None  # the loop's list, to snapshot

    def reset(self, seed=None, options=None):
        obs = np.stack([e.inner.reset()[0] for e in self.envs]).astype(np.int8)
        return obs, {}

    def snapshot(self):
        self.post_states.append(np.stack([np.asarray(e.inner.state, np.int8) for e in self.envs]))
        self.curr_snap.append(list(self.curr_states))

    def step(self, actions):
        if self.steps:
            self.snapshot()  # the loop has finished processing the previous step
        actions = np.asarray(actions)
        obs = np.zeros((self.num_envs, self.single_observation_space.shape[0]), np.int8)
        rew = np.zeros(self.num_envs, np.float64)
        term = np.zeros(self.num_envs, bool)
        trunc = np.zeros(self.num_envs, bool)
        infos = {}
        for i, (e, a) in enumerate(zip(self.envs, actions)):
            o, r, d, t, info = e.inner.step(a)
            if d or t:
                old_o, old_info = o, info
                o, info = e.inner.reset()
                info = dict(info)
                info["final_observation"] = old_o
                info["final_info"] = old_info
            obs[i], rew[i], term[i], trunc[i] = o, r, d, t
            for k, v in info.items():  # SyncVectorEnv._add_info
                if k not in infos:
                    infos[k] = np.full(self.num_envs, None, dtype=object)
                    infos["_" + k] = np.zeros(self.num_envs, bool)
                infos[k][i] = v
                infos["_" + k][i] = True
        self.steps.append(dict(actions=actions.astype(np.int64).copy(), reward=rew.copy(), done=term.copy(),
                               truncated=trunc.copy()))
        return obs, rew, term, trunc, infos


class ScriptedAgent:
    """Uniform random moves (seeded) that ACMove accepts; differentiable dummy heads."""

    def __init__(self, ref, vec, seed):
        import torch
        from torch import nn

        class Heads(nn.Module):
            def __init__(self):
                super().__init__()
                self.logit = nn.Parameter(torch.zeros(12))
                self.v = nn.Parameter(torch.zeros(1))

        self.torch = torch
        self.heads = Heads()
        self.ref, self.vec = ref, vec
        self.rng = np.random.default_rng(seed)
        self.critic = self.actor = self.heads

    def parameters(self):
        return self.heads.parameters()

    def _ok(self, env, a):
        st = np.copy(env.state)
        try:
            self.ref.moves.ACMove(int(a), st, env.max_relator_length, list(env.lengths))
            return True
        except AssertionError:
            return False

    def get_action_and_value(self, x, action=None):
        torch = self.torch
        n = x.shape[0]
        if action is None:
            acts = []
            for e in self.vec.envs:
                while True:
                    a = int(self.rng.integers(0, 12))
                    if self._ok(e.inner, a):
                        break
                acts.append(a)
            action = torch.tensor(acts, dtype=torch.int64)
        logits = self.heads.logit.expand(n, 12)
        dist = torch.distributions.Categorical(logits=logits)
        return action, dist.log_prob(action), dist.entropy(), self.heads.v.expand(n, 1)

    def get_value(self, x):
        return self.heads.v.expand(x.shape[0], 1)


def run_case(ref, initial_states, num_envs, horizon, num_steps, updates, seed, repeat_solved_prob):
    import torch
    vec = RecVecEnv(ref, initial_states, num_envs, horizon)
    agent = ScriptedAgent(ref, vec, seed + 1000)
    optimizer = torch.optim.Adam(agent.parameters(), lr=1e-3)
    curr_states = list(range(num_envs))
    states_processed = set(curr_states)
    success_record = {"solved": set(), "unsolved": set(range(len(initial_states)))}
    ACMoves_hist = {}
    vec.curr_states = curr_states
    batch = num_envs * num_steps
    args = types.SimpleNamespace(
        num_steps=num_steps, num_envs=num_envs, total_timesteps=batch * updates, batch_size=batch,
        minibatch_size=batch // 2, update_epochs=1, seed=seed, anneal_lr=False, is_loss_clip=True, beta=None,
        exp_name="golden", nodes_counts=[8], wandb_log=False, norm_rewards=False, horizon_length=horizon,
        gamma=0.99, gae_lambda=0.95, norm_adv=True, clip_coef=0.2, clip_vloss=True, ent_coef=0.01, vf_coef=0.5,
        max_grad_norm=0.5, target_kl=None, repeat_solved_prob=repeat_solved_prob, lr_decay="linear",
        warmup_period=0.0, learning_rate=1e-3, min_lr_frac=0.0)
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as td:
        os.chdir(td)
        try:
            ref.training.ppo_training_loop(vec, args, "cpu", optimizer, agent, curr_states, success_record,
                                           ACMoves_hist, states_processed, initial_states)
        finally:
            os.chdir(cwd)
    vec.snapshot()  # after the last step
    T = len(vec.steps)
    assert T == num_steps * updates, T
    arr = lambda k, dt: np.stack([s[k] for s in vec.steps]).astype(dt)  # noqa: E731
    return dict(
        initial_states=np.stack(initial_states).astype(np.int8),
        actions=arr("actions", np.int8), reward=arr("reward", np.int32), done=arr("done", np.uint8),
        truncated=arr("truncated", np.uint8), post_state=np.stack(vec.post_states).astype(np.int8),
        curr_states=np.asarray(vec.curr_snap, np.int32),
    ), dict(
        num_envs=num_envs, horizon=horizon, num_steps=num_steps, updates=updates, seed=seed,
        repeat_solved_prob=repeat_solved_prob, solved=sorted(success_record["solved"]),
        unsolved=sorted(success_record["unsolved"]), states_processed=sorted(states_processed),
        ACMoves_hist={str(k): [int(a) for a in v] for k, v in ACMoves_hist.items()},
    )


def cases(ref, ms):
    L = 36

    def pad(r0, r1):
        return ref.utils.convert_relators_to_presentation(r0, r1, L)

    easy = [pad([1], [2, 1]), pad([2], [1, 2]), pad([1, 2], [2]), pad([-1], [2, -1]), pad([1], [-2, 1]),
            pad([2, 1], [1]), pad([1, 2, -1], [2, 2, 1]), pad([2], [1, 1, 2])]
    out = []
    # (a) Miller-Schupp starts + a few that are one or two moves from trivial: round 1 completes,
    # round-2 draws mix solved and unsolved states (repeat_solved_prob 0.25)
    init = []
    for i in range(30):
        if i % 4 == 1:
            init.append(np.asarray(easy[(i // 4) % len(easy)], np.int8))
        else:
            p = ms[i % len(ms)]
            init.append(np.asarray(pad([int(v) for v in p[:18] if v], [int(v) for v in p[18:] if v]), np.int8))
    out.append(("ms_mixed", run_case(ref, init, num_envs=12, horizon=8, num_steps=20, updates=4, seed=3,
                                     repeat_solved_prob=0.25)))
    # (b) mostly easy starts: many solves, round 2 dominated by solved/unsolved choice
    init2 = [np.asarray(easy[i % len(easy)], np.int8) if i % 3 else np.asarray(init[i], np.int8) for i in range(20)]
    out.append(("easy_heavy", run_case(ref, init2, num_envs=8, horizon=5, num_steps=16, updates=5, seed=11,
                                       repeat_solved_prob=0.6)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    a = ap.parse_args()
    ref = load_training(a.reference)
    ms = np.load(os.path.join(HERE, "..", "..", "ac-solver-caltech_amd", "acx", "data", "all_presentations.npy"))
    arrays, meta = {}, {}
    for name, (arr, m) in cases(ref, ms):
        for k, v in arr.items():
            arrays[f"{name}__{k}"] = v
        meta[name] = m
        print(name, "steps", arr["done"].shape, "done", int(arr["done"].sum()), "trunc", int(arr["truncated"].sum()),
              "solved", len(m["solved"]), "processed", len(m["states_processed"]))
    np.savez_compressed(os.path.join(HERE, "curriculum.npz"), **arrays)
    with open(os.path.join(HERE, "curriculum.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
