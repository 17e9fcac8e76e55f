"""ACEnvConfig / ACEnv with the reference's API (ac_solver/envs/ac_env.py), GPU-backed,
plus VecACEnv, the batched environment the MI355X design is built around.

ACEnv      one env; state lives on the device as a (1, 2L) int32 tensor, `step` returns
           numpy like the reference (one acx_step launch + one device->host copy).
VecACEnv   B envs; state (B, 2L) int32 on the device; `step` is one acx_step launch with
           same-step autoreset to each env's starting state (the contract gymnasium's
           SyncVectorEnv gives the reference's PPO loop, environment.py:96-101,
           training.py:238-240); `rollout(T)` is T fused steps in one launch.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional, Union

import numpy as np
import torch

from .. import _lib, ops
from .ac_moves import in_packed_domain, raise_for_err
from .utils import is_array_valid_presentation


class Discrete:
    """Minimal stand-in for gymnasium.spaces.Discrete (gymnasium is not a dependency)."""

    def __init__(self, n: int):
        self.n = n

    def sample(self, rng=None):
        rng = rng or np.random.default_rng()
        return int(rng.integers(self.n))


class Box:
    """Minimal stand-in for gymnasium.spaces.Box."""

    def __init__(self, low, high, dtype=np.int8):
        self.low, self.high, self.dtype = np.asarray(low), np.asarray(high), dtype
        self.shape = self.low.shape


@dataclass
class ACEnvConfig:
    """ac_env.py:14-49 (same fields, defaults and validation)."""

    initial_state: Union[np.ndarray, list] = field(default_factory=lambda: np.array([1, 0, 2, 0]))
    horizon_length: int = 1000
    use_supermoves: bool = False

    def __post_init__(self):
        if isinstance(self.initial_state, list):
            self.initial_state = np.array(self.initial_state)
        if not isinstance(self.initial_state, np.ndarray):
            raise TypeError("initial_state must be a numpy array")
        if self.initial_state.ndim != 1:
            raise ValueError("initial_state must be a 1-dimensional array")
        if len(self.initial_state) % 2 != 0:
            raise ValueError("initial state must have even length")
        if not is_array_valid_presentation(self.initial_state):
            raise ValueError("initial state must be a valid presentation")

    @property
    def max_relator_length(self):
        return len(self.initial_state) // 2

    @classmethod
    def from_dict(cls, config_dict):
        return cls(
            initial_state=np.array(config_dict.get("initial_state", cls().initial_state)),
            horizon_length=config_dict.get("horizon_length", cls().horizon_length),
            use_supermoves=config_dict.get("use_supermoves", cls().use_supermoves),
        )


def _invalid_rows(states: np.ndarray) -> np.ndarray:
    """Vectorised is_array_valid_presentation over (B, 2L) rows (utils.py:13-54)."""
    L = states.shape[1] // 2
    bad = np.zeros(states.shape[0], bool)
    idx = np.arange(L)[None, :]
    for h in range(2):
        nz = states[:, h * L : (h + 1) * L] != 0
        n = nz.sum(1)
        bad |= (n == 0) | (nz & (idx >= n[:, None])).any(1)
    return bad


def _check_domain(state: np.ndarray) -> None:
    if np.any(np.abs(state) > 2):
        raise ValueError("acx presentations use letters +-1 (x) and +-2 (y) only")


class ACEnv:
    """ac_env.py:52-132 on the GPU.  `device` selects the ROCm device (default cuda)."""

    def __init__(self, config: ACEnvConfig = None, device=None):
        config = config if config is not None else ACEnvConfig()
        self.n_gen = 2
        self.max_relator_length = config.max_relator_length
        self.initial_state = config.initial_state
        self.horizon_length = config.horizon_length
        if config.use_supermoves:
            raise NotImplementedError("ACEnv with supermoves is not yet implemented in this library.")
        L = self.max_relator_length
        self.observation_space = Box(np.full(2 * L, -self.n_gen, np.int8), np.full(2 * L, self.n_gen, np.int8))
        self.action_space = Discrete(12)
        self.max_reward = self.horizon_length * self.max_relator_length * self.n_gen
        self.device = torch.device(device if device is not None else "cuda")
        self._dtype = self.initial_state.dtype
        dev = self.device
        # one int32 device block holds everything a step returns -- state 2L | lengths 2 | reward |
        # done, truncated, err as bytes of one slot -- so a step is one launch plus one D2H copy
        # into a pinned host block (no per-step allocations or conversion kernels)
        self._blk = torch.zeros(2 * L + 4, dtype=torch.int32, device=dev)
        self._host = torch.empty(2 * L + 4, dtype=torch.int32, pin_memory=True)
        b8 = self._blk.view(torch.uint8)
        self._state = self._blk[: 2 * L].view(1, 2 * L)
        self._lens = self._blk[2 * L : 2 * L + 2].view(1, 2)
        self._reward = self._blk[2 * L + 2 : 2 * L + 3]
        self._done = b8[4 * (2 * L + 3) : 4 * (2 * L + 3) + 1]
        self._trunc = b8[4 * (2 * L + 3) + 1 : 4 * (2 * L + 3) + 2]
        self._err = b8[4 * (2 * L + 3) + 2 : 4 * (2 * L + 3) + 3]
        self._action = torch.empty((1,), dtype=torch.int32, device=dev)
        self._count = torch.zeros((1,), dtype=torch.int32, device=dev)
        self._set_state(np.copy(self.initial_state))
        self.actions = []

    def _set_state(self, state: np.ndarray) -> None:
        L = self.max_relator_length
        self.state = np.asarray(state)
        # letters +-1/+-2 with zeros only as right padding: the packed step kernel (acx_step);
        # anything else the reference accepts (other integer letters): the exact word kernel
        self._packed = in_packed_domain(self.state, L)
        self._state.copy_(torch.as_tensor(self.state.astype(np.int32)).reshape(1, 2 * L))
        self.lengths = [int(np.count_nonzero(self.state[i * L : (i + 1) * L])) for i in range(self.n_gen)]
        self.count_steps = 0
        self._count.zero_()

    @property
    def state_tensor(self) -> torch.Tensor:
        """The (1, 2L) int32 device tensor backing the env."""
        return self._state

    def step(self, action):
        self.actions += [action]
        self._action.fill_(int(action))
        if not self._packed:
            return self._step_words()
        ops.step(self._state, self._action, state_out=self._state, step_count=self._count,
                 horizon=self.horizon_length, cyclical=True, reward=self._reward, done=self._done,
                 truncated=self._trunc, lengths=self._lens, err=self._err)
        L = self.max_relator_length
        self._host.copy_(self._blk, non_blocking=True)
        torch.cuda.current_stream(self.device).synchronize()
        h = self._host.numpy()
        flags = int(h[2 * L + 3])  # little-endian bytes: done, truncated, err
        raise_for_err((flags >> 16) & 0xff, "ACEnv.step")
        self.state = h[: 2 * L].astype(self._dtype)
        self.lengths = [int(h[2 * L]), int(h[2 * L + 1])]
        reward, done, truncated = int(h[2 * L + 2]), bool(flags & 0xff), bool((flags >> 8) & 0xff)
        self.count_steps += 1
        return self.state, reward, done, truncated, ({"actions": self.actions.copy()} if done else {})

    def _step_words(self):
        """ac_env.py:91-111 for states outside the packed domain: acx_word_move (ACMove with
        cyclical=True, exact on any integer letters) + the env's reward / truncation bookkeeping."""
        L = self.max_relator_length
        out, lens, done, err = ops.word_move(self._state, self._action, cyclical=True)
        host = torch.cat([out.reshape(-1), lens.reshape(-1), done.to(torch.int32), err.to(torch.int32)]).cpu().numpy()
        raise_for_err(int(host[-1]), "ACEnv.step")
        self._state.copy_(out)
        self.state = host[: 2 * L].astype(self._dtype)
        self.lengths = [int(host[2 * L]), int(host[2 * L + 1])]
        done = bool(host[2 * L + 2])
        reward = self.max_reward * done - sum(self.lengths) * (1 - done)
        self.count_steps += 1
        truncated = self.count_steps >= self.horizon_length
        return self.state, reward, done, truncated, ({"actions": self.actions.copy()} if done else {})

    def reset(self, *, seed=None, options=None):
        start = options["starting_state"] if options and "starting_state" in options else self.initial_state
        start = np.copy(start)
        self._set_state(start)
        self.actions = []
        return self.state, {}

    def render(self):
        pass

    @property
    def unwrapped(self):
        return self


def _row_extent(rows: torch.Tensor, L: int) -> torch.Tensor:
    """(B, 2) int32: per relator, the position after its last non-zero letter -- its length for
    a canonical row; for any other row (a gap, a letter out of domain) it still covers every
    non-zero entry, so acx_step_lengths reads them and reports the row as acx_step would"""
    nz = rows.reshape(-1, 2, L) != 0
    pos = torch.arange(1, L + 1, dtype=torch.int32, device=rows.device)
    return (nz * pos).amax(dim=2).to(torch.int32)


class VecACEnv:
    """B Andrews-Curtis envs stepped by one kernel launch per step.

    initial_states: (B, 2L) array/tensor of starting presentations (each env resets to its
    own row).  All buffers live on `device`; `step` takes a (B,) int32 device tensor of
    move ids and returns device tensors (obs, reward, done, truncated, info) where obs is
    the post-autoreset state and info["final_observation"] holds, for rows with
    done | truncated, the state before the reset.

    record_actions=True keeps each env's episode moves on the device (acx_step_record) and
    fills the info dict the PPO trainer reads for solved episodes (training.py:273-280), as
    gymnasium's SyncVectorEnv builds it from ACEnv's per-env info (ac_env.py:105-110):
      info_format "final_info" (gymnasium < 1.0, same-step autoreset): info["final_info"] is an
        object array with {"actions": [...]} for done envs, {} for truncated ones, None else,
        info["_final_info"] / info["_final_observation"] the finished mask;
      info_format "actions" (the gymnasium >= 1.0 key layout): info["actions"][i] = the move list
        of env i's solved episode, info["_actions"] its mask.
    Building it synchronises with the device once per step (the trainer reads it on the host).

    autoreset_mode "same_step" (default; gymnasium < 1.0, what the reference trains with): the
    step that ends an episode returns the env's starting state.  "next_step" (gymnasium >= 1.0):
    it returns the terminal state, and the env's next step resets it instead of moving (action
    ignored, reward 0, done = truncated = False) -- acx_step_next; its info layout is "actions"
    (no final_observation).  Parity unpinned: gymnasium is an un-vendored dependency.
    """

    def __init__(self, initial_states, horizon_length: int = 1000, device=None, cyclical: bool = True,
                 track_final_obs: bool = True, check_errors: bool = False, record_actions: bool = False,
                 info_format: str = "final_info", autoreset_mode: str = "same_step"):
        self.device = torch.device(device if device is not None else "cuda")
        init = torch.as_tensor(np.asarray(initial_states) if not torch.is_tensor(initial_states) else initial_states)
        if init.dim() != 2 or init.shape[1] % 2:
            raise ValueError("initial_states must be (B, 2L)")
        init_np = init.cpu().numpy()
        bad = _invalid_rows(init_np)
        if bad.any():
            raise ValueError(f"initial state {init_np[np.argmax(bad)]} is not a valid presentation")
        _check_domain(init_np)
        self.num_envs = init.shape[0]
        self.max_relator_length = init.shape[1] // 2
        self.horizon_length = int(horizon_length)
        self.cyclical = bool(cyclical)
        self.check_errors = check_errors
        B, L, dev = self.num_envs, self.max_relator_length, self.device
        self.max_reward = self.horizon_length * L * 2
        self.reset_state = init.to(dev, torch.int32).contiguous()
        self.state = self.reset_state.clone()
        self.step_count = torch.zeros(B, dtype=torch.int32, device=dev)
        self.reward = torch.empty(B, dtype=torch.int32, device=dev)
        self.done = torch.empty(B, dtype=torch.uint8, device=dev)
        self.truncated = torch.empty(B, dtype=torch.uint8, device=dev)
        # the rows' relator lengths: kept current so that a plain step reads and writes only the
        # letters (acx_step_lengths); _lengths_ok is False after anything that changed rows without
        # them (rollout, direct writes by a learner), and the next step uses acx_step, which rewrites them
        self.lengths = _row_extent(self.state, L).contiguous()
        self._lengths_ok = True
        # per row: the previous lengths-carrying step left both relators reduced (bit 0 freely, bit 1
        # cyclically; 0 unknown) -- acx_step_lengths_reduced then leaves a conjugation's other
        # relator unread.  _reduced_ok is False after a step by any other kernel (which does not
        # write the flags); the next lengths-carrying step zeroes them first
        self.reduced = torch.zeros(B, dtype=torch.uint8, device=dev)
        self._reduced_ok = True
        # the lengths-carrying step where it measured faster (ops.lengths_step_for: L = 128, and L = 36
        # above the small-batch range)
        self._live_tile = ops.lengths_step_for(B, L)
        self.err = torch.zeros(B, dtype=torch.uint8, device=dev)
        self.err_count = torch.zeros(1, dtype=torch.int32, device=dev)
        if autoreset_mode not in ("same_step", "next_step"):
            raise ValueError("autoreset_mode must be 'same_step' or 'next_step'")
        self.autoreset_mode = autoreset_mode
        if autoreset_mode == "next_step":
            if record_actions and info_format != "actions":
                raise ValueError("autoreset_mode='next_step' reports info in the 'actions' layout (gymnasium >= 1.0)")
            track_final_obs = False  # the ending step's own observation is the terminal state
            self.pending = torch.zeros(B, dtype=torch.uint8, device=dev)
        self.final_obs = torch.zeros_like(self.state) if track_final_obs else None
        if info_format not in ("final_info", "actions"):
            raise ValueError("info_format must be 'final_info' or 'actions'")
        self.record_actions = bool(record_actions)
        self.info_format = info_format
        if self.record_actions:
            # move k of env i's current episode at [(hist_base[i] + k) mod H, i] (a ring, step-major:
            # a step's moves go to one row however far apart the episodes are, acx.h); an episode
            # never outlives the horizon
            self.action_hist = torch.zeros((max(1, self.horizon_length), B), dtype=torch.uint8, device=dev)
            self.hist_base = torch.zeros(B, dtype=torch.int32, device=dev)
            self.hist_t = 0  # steps taken: the ring row of this step's moves
            self.episode_len = torch.zeros(B, dtype=torch.int32, device=dev)
        self.action_space = Discrete(12)
        self.single_observation_space = Box(np.full(2 * L, -2, np.int8), np.full(2 * L, 2, np.int8))

    def reset(self, *, seed=None, options=None):
        """Reset every env to its starting state (options["starting_states"] replaces them).
        Like the reference's ACEnv.reset (ac_env.py:113-129) the rows are taken as they are, with
        no validation: a row outside the packed domain (a zero inside a relator, a letter other
        than +-1/+-2) is held as its exact values and every step reports it with err 3
        (ACX_ERR_DOMAIN), as the step kernels do for such starting rows."""
        if options and "starting_states" in options:
            rows = np.asarray(options["starting_states"]).reshape(tuple(self.reset_state.shape))
            self.reset_state.copy_(torch.as_tensor(rows.astype(np.int32)).to(self.device))
        self.state.copy_(self.reset_state)
        # (reset_state may also have been rewritten on the device, e.g. by the learner's curriculum)
        self.lengths.copy_(_row_extent(self.state, self.max_relator_length))
        self._lengths_ok = True
        self.reduced.zero_()
        self._reduced_ok = True
        self.step_count.zero_()
        if self.autoreset_mode == "next_step":
            self.pending.zero_()
        return self.state, {}

    def reset_env(self, i: int, starting_state) -> None:
        """envs.envs[i].reset(options={"starting_state": s}) (training.py:351-352): env i now
        starts (and later autoresets) from `starting_state`."""
        s = np.asarray(starting_state)
        if not is_array_valid_presentation(s):
            raise ValueError("starting_state must be a valid presentation")
        _check_domain(s)
        t = torch.as_tensor(s.astype(np.int32), device=self.device)
        self.reset_state[i].copy_(t)
        self.state[i].copy_(t)
        self.lengths[i].copy_(_row_extent(t, self.max_relator_length)[0])
        self.reduced[i] = 0
        self.step_count[i] = 0
        if self.autoreset_mode == "next_step":
            self.pending[i] = 0

    def _step_args(self):
        """Pointers of the env's persistent buffers, computed once (the per-call Python
        overhead of argument checking would otherwise rival a small batch's kernel time)."""
        if getattr(self, "_args", None) is None:
            fo = self.final_obs.data_ptr() if self.final_obs is not None else None
            self._args = (self.state.data_ptr(), self.state.data_ptr(), self.reset_state.data_ptr(),
                          self.step_count.data_ptr(), self.reward.data_ptr(), self.done.data_ptr(),
                          self.truncated.data_ptr(), self.lengths.data_ptr(), fo, self.err.data_ptr(),
                          self.err_count.data_ptr())
            self._lib = _lib.load()
        return self._args

    def step(self, actions: torch.Tensor):
        if (actions.dtype != torch.int32 or actions.device != self.device or not actions.is_contiguous()
                or actions.shape != (self.num_envs,)):
            actions = actions.to(self.device, torch.int32).contiguous().reshape(self.num_envs)
        s_in, s_out, rs, cnt, rew, dn, tr, ln, fo, err, ec = self._step_args()
        stream = ops._stream(self.device)
        live = (self.autoreset_mode != "next_step" and self._lengths_ok and self._live_tile
                and not self.record_actions)
        if self.autoreset_mode == "next_step":
            rec = self.record_actions
            st = self._lib.acx_step_next(s_in, s_out, actions.data_ptr(), rs, cnt, rew, dn, tr, ln,
                                         self.pending.data_ptr(), self.action_hist.data_ptr() if rec else None,
                                         self.action_hist.shape[0] if rec else 0,
                                         self.hist_base.data_ptr() if rec else None, self.hist_t if rec else 0,
                                         self.episode_len.data_ptr() if rec else None, err, ec, self.num_envs,
                                         self.max_relator_length, self.horizon_length, int(self.cyclical), stream)
            _lib.check(st, "acx_step_next")
        elif live:
            # the rows' lengths are current: only their letters are read and written (and of a
            # reduced row only the relator a conjugation changes)
            if not self._reduced_ok:
                self.reduced.zero_()
                self._reduced_ok = True
            st = self._lib.acx_step_lengths_reduced(s_in, actions.data_ptr(), rs, cnt, rew, dn, tr, ln,
                                                    self.reduced.data_ptr(), fo, err, ec, self.num_envs,
                                                    self.max_relator_length, self.horizon_length,
                                                    int(self.cyclical), stream)
            _lib.check(st, "acx_step_lengths_reduced")
        elif self.record_actions:
            st = self._lib.acx_step_record(s_in, s_out, actions.data_ptr(), rs, cnt, rew, dn, tr, ln, fo,
                                           self.action_hist.data_ptr(), self.action_hist.shape[0],
                                           self.hist_base.data_ptr(), self.hist_t, self.episode_len.data_ptr(),
                                           err, ec, self.num_envs,
                                           self.max_relator_length, self.horizon_length, int(self.cyclical), stream)
            _lib.check(st, "acx_step_record")
        else:
            st = self._lib.acx_step(s_in, s_out, actions.data_ptr(), rs, cnt, rew, dn, tr, ln, fo, err, ec,
                                    self.num_envs, self.max_relator_length, self.horizon_length, int(self.cyclical),
                                    stream)
            _lib.check(st, "acx_step")
        self._lengths_ok = True  # every step kernel writes the rows' lengths
        self._reduced_ok = live  # ... only the lengths-carrying one the reduced flags
        if self.record_actions:
            self.hist_t += 1
        if self.check_errors:
            self.raise_if_errors()
        info = {"final_observation": self.final_obs} if self.final_obs is not None else {}
        if self.record_actions:
            info.update(self._episode_info())
        return self.state, self.reward, self.done, self.truncated, info

    def _episode_info(self) -> dict:
        """SyncVectorEnv's info entries for the envs whose episode ended this step (one D2H copy
        of the masks, then one column of the move history per solved env)."""
        B = self.num_envs
        flags = torch.stack([self.done, self.truncated]).cpu().numpy().astype(bool)
        done, fin = flags[0], flags[0] | flags[1]
        if not fin.any():  # SyncVectorEnv adds the keys only when some env finished
            return {}
        solved = np.flatnonzero(done)
        lists = {}
        if solved.size:
            idx = torch.as_tensor(solved, device=self.device)
            lens = self.episode_len[idx].cpu().numpy()
            n_max = int(lens.max())
            rows = (self.hist_base[idx].to(torch.int64)[None, :] +
                    torch.arange(n_max, dtype=torch.int64, device=self.device)[:, None]) % self.action_hist.shape[0]
            cols = self.action_hist[rows, idx[None, :]].cpu().numpy()  # (max_len, n_solved)
            lists = {int(i): [int(a) for a in cols[: lens[k], k]] for k, i in enumerate(solved)}
        if self.info_format == "final_info":
            final_info = np.full(B, None, dtype=object)
            for i in np.flatnonzero(fin):
                final_info[i] = {"actions": lists[int(i)]} if done[i] else {}
            return {"final_info": final_info, "_final_info": fin, "_final_observation": fin}
        acts = np.full(B, None, dtype=object)
        for i, v in lists.items():
            acts[i] = v
        return {"actions": acts, "_actions": done}

    def rollout(self, actions: torch.Tensor, obs_traj: Optional[torch.Tensor] = None, reward_traj=None,
                done_traj=None, trunc_traj=None):
        """T = actions.shape[0] steps in one launch; trajectories optional (T, B, ...).  obs_traj
        is int32, or int8 -- the observation_space dtype (ac_env.py:64-70) and what
        SyncVectorEnv returns -- at a quarter of the bytes.

        Same-step autoreset only: the fused rollout resets an env on the step its episode ends.
        With autoreset_mode="next_step" (acx_step_next's pending flags) or record_actions (the
        per-episode move history acx_step_record keeps) a rollout would leave that per-env state
        stale, so it raises instead."""
        if self.autoreset_mode == "next_step":
            raise ValueError("VecACEnv.rollout implements same-step autoreset only; with autoreset_mode='next_step' "
                             "step the env with step()")
        if self.record_actions:
            raise ValueError("VecACEnv.rollout does not record episode moves; with record_actions=True step the env "
                             "with step()")
        ops.rollout(self.state, actions, self.reset_state, self.step_count, horizon=self.horizon_length,
                    cyclical=self.cyclical, obs_traj=obs_traj, reward_traj=reward_traj, done_traj=done_traj,
                    trunc_traj=trunc_traj, err=self.err, err_count=self.err_count)
        self._lengths_ok = False  # the rollout does not write lengths
        self._reduced_ok = False
        if self.check_errors:
            self.raise_if_errors()

    def raise_if_errors(self) -> None:
        n = int(self.err_count.item())
        if n:
            codes = self.err[self.err != 0]
            raise_for_err(int(codes[0].item()), f"VecACEnv ({n} env(s) failed)")
