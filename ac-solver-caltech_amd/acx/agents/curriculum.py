"""Host half of the PPO start-state curriculum (ac_solver/agents/training.py:264-352).

LearnerEnv keeps the per-step env work and the round-1 curriculum on the GPU (finished envs
take `max(states_processed) + 1` in env order, :329-336).  What stays on the host is what the
reference keeps in Python containers and draws with Python `random`:

  * success_record {"solved", "unsolved"} sets and ACMoves_hist, updated for every solved
    episode from its info["actions"] list (:267-292);
  * after round 1, the random restart choice (:337-348): an unsolved state when nothing is
    solved yet, or with probability 1 - repeat_solved_prob; else a solved one --
    `random.uniform(0, 1)` and `random.choice(list(<set>))` on the same sets, in the same order
    and with the same short-circuit, so a caller that seeds `random` like the trainer
    (`random.seed(args.seed + update)`, :203-204) draws the reference's states;
  * curr_states / states_processed (:319-350).

Envs are processed in env order, a solved episode's bookkeeping before its own restart choice,
exactly as the reference's loop over `_record_info` does.
"""

from __future__ import annotations

import random as _random

import numpy as np


class CurriculumRecord:
    def __init__(self, n_states: int, num_envs: int, repeat_solved_prob: float, rng=None):
        self.n_states = int(n_states)
        self.repeat_solved_prob = float(repeat_solved_prob)
        self.rng = rng if rng is not None else _random  # the trainer's global `random` by default
        # environment.py:96-110
        self.curr_states = list(range(num_envs))
        self.states_processed = set(self.curr_states)
        self.success_record = {"solved": set(), "unsolved": set(range(self.n_states))}
        self.ACMoves_hist = {}

    def on_done(self, i: int, action_list) -> bool:
        """Env i's episode (started from curr_states[i]) was solved with `action_list`
        (training.py:267-292).  Returns True if it is a new best path for that state."""
        c = self.curr_states[i]
        if c in self.success_record["unsolved"]:
            self.success_record["unsolved"].remove(c)
            self.success_record["solved"].add(c)
        prev = self.ACMoves_hist.get(c)
        if prev is None or len(action_list) < len(prev):
            self.ACMoves_hist[c] = list(action_list)
            return True
        return False

    def draw(self) -> int:
        """The restart choice after round 1 (training.py:339-348)."""
        solved, unsolved = self.success_record["solved"], self.success_record["unsolved"]
        if len(solved) == 0 or (unsolved and self.rng.uniform(0, 1) > self.repeat_solved_prob):
            return self.rng.choice(list(unsolved))
        return self.rng.choice(list(solved))

    def restart(self, i: int, k: int) -> None:
        """Env i restarts from initial state k (training.py:350-352)."""
        self.curr_states[i] = int(k)
        self.states_processed.add(int(k))

    def process(self, env, done, truncated, needs_host, obs_out=None) -> list:
        """One step's bookkeeping next to LearnerEnv.step: `done`, `truncated`, `needs_host` as
        returned by it (device or host arrays).  Solved episodes update the record from
        env.episode_actions_many (one copy for all of them); envs the device placed (round 1) take env.curr_index[i]; envs it
        flagged are drawn here and placed with env.place (obs_out: the step's observation row
        buffer, as for LearnerEnv.place).  Returns [(env, state index)] for every restart."""
        if hasattr(env, "failed") and env.failed():
            raise RuntimeError("LearnerEnv: a curriculum ranking gave up (acx_learner_step's sticky failure word: "
                               "needs_host 3 or a stale next_index); call env.reset_workspace() before stepping on")
        d = np.asarray(done.cpu() if hasattr(done, "cpu") else done).astype(bool)
        t = np.asarray(truncated.cpu() if hasattr(truncated, "cpu") else truncated).astype(bool)
        fin = np.nonzero(d | t)[0]
        if fin.size == 0:
            return []
        dev_idx = env.curr_index.cpu().numpy()
        # the solved episodes' move lists, copied to the host together (one transfer per step)
        solved = [i for i in fin.tolist() if d[i]]
        if hasattr(env, "episode_actions_many"):
            acts = env.episode_actions_many(solved)
        else:
            acts = {i: env.episode_actions(i) for i in solved}
        out = []
        hv = np.asarray(needs_host.cpu() if hasattr(needs_host, "cpu") else needs_host)
        if (hv == 3).any():
            raise RuntimeError("LearnerEnv: the device could not rank the finished envs (needs_host 3: a ranking wait "
                               "gave up); call env.reset_workspace() before stepping on")
        for i in fin.tolist():
            if d[i]:
                self.on_done(i, acts[i])
            if hv[i] == 1:  # round 1 complete: the reference's random draw (training.py:337-348)
                k = self.draw()
                env.place(i, k, obs_out=obs_out)
            else:
                k = int(dev_idx[i])
            self.restart(i, k)
            out.append((i, k))
        return out
