"""Device-resident env plumbing for the PPO rollout phase (ac_solver/agents/training.py:221-356).

The reference steps a gymnasium SyncVectorEnv on the host each step (`envs.step(action.cpu()
.numpy())`, training.py:238-240), copies obs/reward/done back to the device (:241, :354-356)
and runs a Python loop over the envs for episode bookkeeping and the start-state curriculum
(:262-352).  LearnerEnv keeps all of it on the GPU, one acx_learner_step call -- ONE kernel
launch, the curriculum's ranking fused into the step -- per step:

  * the policy's int64 actions go straight in;
  * the next observation is written as float32 into whatever (B, 2L) buffer the caller names
    (e.g. obs[t + 1] of the learner's (T, B, 2L) buffer), rewards[t] and next_done likewise;
  * each env's current episode moves are kept in a (hist_cap, B) byte buffer, so info["actions"]
    of a solved episode (training.py:275-280) is one column read;
  * the round-1 curriculum (training.py:319-336, 349-352) runs on the device: finished envs
    take the next unprocessed initial state in env order.  Once every initial state has been
    used the reference draws random solved/unsolved states with Python `random` (:337-346);
    those envs are flagged in `needs_host` and placed by `place()`.  needs_host 3: the device
    could not rank the env (a ranking wait gave up) -- CurriculumRecord.process raises, as it does
    on the workspace's sticky failure word (`failed()`); `reset_workspace()` recovers.  One
    LearnerEnv's steps must not run concurrently (they share the workspace; unsupported).
"""

from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from .. import _lib, ops
from ..envs.ac_env import VecACEnv


class LearnerEnv:
    def __init__(self, initial_states, num_envs: int, horizon_length: int = 200, device=None,
                 cyclical: bool = True, hist_cap: Optional[int] = None):
        init = np.asarray(initial_states)
        if init.ndim != 2 or num_envs > init.shape[0]:
            raise ValueError("initial_states must be (N, 2L) with N >= num_envs (environment.py:82-86)")
        # env i starts at initial_states[i]; states 0..num_envs-1 are processed (environment.py:96-101)
        self.vec = VecACEnv(init[:num_envs], horizon_length=horizon_length, device=device, cyclical=cyclical,
                            track_final_obs=False)
        dev = self.vec.device
        self.device = dev
        self.num_envs = num_envs
        self.L = self.vec.max_relator_length
        self.horizon_length = int(horizon_length)
        self.initial_states = torch.as_tensor(init.astype(np.int32)).to(dev).contiguous()
        self.n_states = init.shape[0]
        self.curr_index = torch.arange(num_envs, dtype=torch.int32, device=dev)
        self.next_index = torch.tensor([num_envs], dtype=torch.int32, device=dev)  # max(states_processed) + 1
        self.needs_host = torch.zeros(num_envs, dtype=torch.uint8, device=dev)
        self.hist_cap = int(hist_cap if hist_cap is not None else horizon_length)
        # move k of env i's episode at [(hist_base[i] + k) mod hist_cap, i]: a ring, step-major, so
        # every env writes a step's move to one row however far apart the episodes are (acx.h)
        self.action_hist = torch.zeros((self.hist_cap, num_envs), dtype=torch.uint8, device=dev)
        self.hist_base = torch.zeros(num_envs, dtype=torch.int32, device=dev)
        self.hist_t = 0  # steps taken: the ring row of this step's moves
        self.episode_len = torch.zeros(num_envs, dtype=torch.int32, device=dev)
        self.done = torch.zeros(num_envs, dtype=torch.uint8, device=dev)
        self.truncated = torch.zeros(num_envs, dtype=torch.uint8, device=dev)
        self._ws = torch.zeros(int(_lib.load().acx_curriculum_workspace(num_envs)), dtype=torch.int32, device=dev)
        self._fail_word = int(_lib.load().acx_learner_failure_word(num_envs))

    def failed(self) -> bool:
        """True once a ranking of acx_learner_step gave up (acx.h: needs_host 3, or the last tile's
        total never arrived and next_index is stale); every later step ranks nothing until
        reset_workspace().  One small device-to-host copy."""
        return bool(self._ws[self._fail_word: self._fail_word + 2].any().item())

    def reset_workspace(self) -> None:
        """After a failed ranking: re-zero the curriculum workspace and restore next_index in round 1
        (every finished env the device did rank holds its state in curr_index, acx.h)."""
        self._ws.zero_()
        if int(self.next_index.item()) < self.n_states:
            nxt = max(int(self.next_index.item()), int(self.curr_index.max().item()) + 1)
            self.next_index.fill_(min(nxt, self.n_states))

    @property
    def state(self) -> torch.Tensor:
        return self.vec.state

    def initial_obs(self, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """next_obs before the first step (training.py:190-193) as float32."""
        o = self.vec.state.to(torch.float32)
        if out is not None:
            out.copy_(o)
            return out
        return o

    def step(self, action: torch.Tensor, obs_out: Optional[torch.Tensor] = None,
             reward_out: Optional[torch.Tensor] = None, done_out: Optional[torch.Tensor] = None,
             fused: bool = True):
        """One env step for all envs.  action: (B,) int64 (policy samples) or int32 device tensor.
        obs_out / reward_out / done_out: float32 (B, 2L) / (B,) / (B,) device views to fill
        (next_obs, rewards[t], next_done).  Returns (done, truncated, episode_len, needs_host)
        uint8/int32 device tensors; no host synchronisation.  fused (default): one
        acx_learner_step call (one launch); else acx_step_learner + acx_curriculum_assign (four)."""
        lib = _lib.load()
        B, L, dev = self.num_envs, self.L, self.device
        for name, t, shape in (("obs_out", obs_out, (B, 2 * L)), ("reward_out", reward_out, (B,)),
                               ("done_out", done_out, (B,))):
            if t is not None and (t.dtype != torch.float32 or t.shape != shape or t.device != dev
                                  or not t.is_contiguous()):
                raise ValueError(f"{name} must be a contiguous float32 {shape} tensor on {dev}")
        if action.device != dev or action.shape != (B,) or not action.is_contiguous():
            action = action.to(dev).contiguous().reshape(B)
        a32 = action if action.dtype == torch.int32 else None
        a64 = action if action.dtype == torch.int64 else None
        if a32 is None and a64 is None:
            a64 = action.to(torch.int64)
        v = self.vec
        v._lengths_ok = False  # the learner step does not write the vector env's lengths
        stream = ops._stream(dev)
        ptr = lambda t: None if t is None else t.data_ptr()  # noqa: E731
        if fused:
            st = lib.acx_learner_step(
                v.state.data_ptr(), ptr(a32), ptr(a64), v.reset_state.data_ptr(), v.step_count.data_ptr(),
                ptr(obs_out), ptr(reward_out), ptr(done_out), self.done.data_ptr(), self.truncated.data_ptr(),
                self.action_hist.data_ptr(), self.hist_cap, self.hist_base.data_ptr(), self.hist_t,
                self.episode_len.data_ptr(), v.err.data_ptr(), v.err_count.data_ptr(), self.initial_states.data_ptr(),
                self.n_states, self.next_index.data_ptr(), self.curr_index.data_ptr(), self.needs_host.data_ptr(),
                self._ws.data_ptr(), B, L, self.horizon_length, int(v.cyclical), stream)
            _lib.check(st, "acx_learner_step")
            self.hist_t += 1
            return self.done, self.truncated, self.episode_len, self.needs_host
        st = lib.acx_step_learner(
            v.state.data_ptr(), ptr(a32), ptr(a64), v.reset_state.data_ptr(), v.step_count.data_ptr(), ptr(obs_out),
            ptr(reward_out), ptr(done_out), self.done.data_ptr(), self.truncated.data_ptr(),
            self.action_hist.data_ptr(), self.hist_cap, self.hist_base.data_ptr(), self.hist_t,
            self.episode_len.data_ptr(), None, v.err.data_ptr(), v.err_count.data_ptr(), B, L, self.horizon_length,
            int(v.cyclical), stream)
        _lib.check(st, "acx_step_learner")
        self.hist_t += 1
        st = lib.acx_curriculum_assign(
            self.done.data_ptr(), self.truncated.data_ptr(), self.initial_states.data_ptr(), self.n_states,
            self.next_index.data_ptr(), self.curr_index.data_ptr(), self.needs_host.data_ptr(), v.state.data_ptr(),
            v.reset_state.data_ptr(), ptr(obs_out), self._ws.data_ptr(), B, L, stream)
        _lib.check(st, "acx_curriculum_assign")
        return self.done, self.truncated, self.episode_len, self.needs_host

    def episode_actions(self, i: int) -> list:
        """info["actions"] of env i's episode that ended at the last step (training.py:275-280)."""
        return self.episode_actions_many([i])[int(i)]

    def episode_actions_many(self, envs) -> dict:
        """{i: info["actions"]} for the envs `envs` (host ints) whose episodes ended at the last
        step: one copy of their episode lengths and one of their action-history columns (not a
        device round trip per env)."""
        envs = [int(i) for i in envs]
        if not envs:
            return {}
        idx = torch.as_tensor(envs, dtype=torch.int64, device=self.episode_len.device)
        lens = self.episode_len[idx].cpu().numpy()
        n_max = int(lens.max())
        if n_max > self.hist_cap:
            raise ValueError(f"episode of {n_max} moves exceeds hist_cap {self.hist_cap}")
        rows = (self.hist_base[idx].to(torch.int64)[None, :] +
                torch.arange(n_max, dtype=torch.int64, device=idx.device)[:, None]) % self.hist_cap
        cols = self.action_hist[rows, idx[None, :]].cpu().numpy()  # (n_max, len(envs))
        return {i: [int(x) for x in cols[: int(lens[j]), j]] for j, i in enumerate(envs)}

    def place(self, i: int, state_index: int, obs_out: Optional[torch.Tensor] = None) -> None:
        """Host placement of env i (after round 1, training.py:337-352): start from
        initial_states[state_index]."""
        s = self.initial_states[state_index]
        self.vec.reset_state[i].copy_(s)
        self.vec.state[i].copy_(s)
        self.vec._lengths_ok = False
        self.vec.step_count[i] = 0
        self.curr_index[i] = state_index
        self.needs_host[i] = 0
        if obs_out is not None:
            obs_out[i].copy_(s.to(torch.float32))
