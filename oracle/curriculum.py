"""CPU restatement of the env side of the PPO rollout phase (TEST INFRASTRUCTURE ONLY).

Follows ac_solver/agents/training.py:221-352 with the oracle env step (oracle.env_step =
ACEnv.step + SyncVectorEnv same-step autoreset) for one vector of envs:
  * env i starts at initial_states[i], states_processed = {0..B-1} (environment.py:96-101);
  * per step: actions appended to each env's episode list (ac_env.py:96), the episode's list is
    info["actions"] when done (ac_env.py:105, training.py:275-280);
  * for every env with done | truncated, in env order (training.py:262-352): round1_complete
    once max(states_processed) == N - 1 (:329-333); if not complete the env takes
    max(states_processed) + 1 (:334-336), else the caller's `host_pick(i)` stands in for the
    random solved/unsolved draw (:337-346); states_processed gains it; the env restarts from
    initial_states[k] (:349-352)."""

from __future__ import annotations

import numpy as np

from . import oracle as O


class RolloutEnvs:
    def __init__(self, initial_states, num_envs, horizon, cyclical=True):
        self.init = np.asarray(initial_states, np.int32)
        self.L = self.init.shape[1] // 2
        self.H = horizon
        self.cyc = cyclical
        self.state = self.init[:num_envs].copy()
        self.reset_rows = self.init[:num_envs].copy()
        self.count = np.zeros(num_envs, np.int32)
        self.curr_states = list(range(num_envs))
        self.states_processed = set(self.curr_states)
        self.round1_complete = False
        self.episode = [[] for _ in range(num_envs)]

    def step(self, actions, host_pick, on_done=None):
        """on_done(i, action_list): called for a solved env before its restart choice, in env
        order (training.py:267-292 precede :319-352 for the same env)."""
        B = self.state.shape[0]
        for i in range(B):
            self.episode[i].append(int(actions[i]))
        r, d, tr, e, _, _ = O.env_step(self.state, np.asarray(actions, np.int32), self.L, self.H, self.count,
                                       reset_state=self.reset_rows, cyclical=self.cyc)
        assert not e.any()
        info_actions, ep_len, picked_by_host = {}, np.zeros(B, np.int32), np.zeros(B, bool)
        for i in range(B):
            if d[i] or tr[i]:
                ep_len[i] = len(self.episode[i])
                if d[i]:
                    info_actions[i] = list(self.episode[i])
                    if on_done is not None:
                        on_done(i, info_actions[i])
                self.episode[i] = []
                self.round1_complete = self.round1_complete or max(self.states_processed) == len(self.init) - 1
                if not self.round1_complete:
                    k = max(self.states_processed) + 1
                else:
                    k = host_pick(i)
                    picked_by_host[i] = True
                self.curr_states[i] = k
                self.states_processed.add(k)
                self.state[i] = self.init[k]
                self.reset_rows[i] = self.init[k]
                self.count[i] = 0
        return dict(reward=r, done=d, truncated=tr, episode_len=ep_len, info_actions=info_actions,
                    picked_by_host=picked_by_host)
