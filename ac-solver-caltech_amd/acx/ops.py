"""Torch-facing wrappers of the libacx.so kernels (include/acx.h).

Every function takes/returns torch tensors on a ROCm device, launches on the current
torch stream and never synchronises.  Presentations are (B, 2L) int32 tensors.
"""

from __future__ import annotations

from typing import Optional

import torch

from . import _lib

_INT32 = torch.int32
_UINT8 = torch.uint8


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _stream(device: torch.device) -> int:
    """The raw handle of `device`'s current stream.  torch's own getter of the raw handle takes
    ~0.08 us; torch.cuda.current_stream(device).cuda_stream builds a Stream object first (~1.8 us,
    tools/host_overhead.py) -- a fifth of a per-call step's host path, whose kernel at 65,536 envs
    is ~10 us."""
    if _RAW_STREAM is not None:
        return _RAW_STREAM(device.index if device.index is not None else torch.cuda.current_device())
    return torch.cuda.current_stream(device).cuda_stream


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _need_gpu(t: torch.Tensor, name: str) -> None:
    if not t.is_cuda:
        raise _lib.ACXError(f"{name} must be a ROCm device tensor (acx has no CPU path)")


def _check(t: Optional[torch.Tensor], name: str, dtype: torch.dtype, shape, device) -> None:
    if t is None:
        return
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name}: expected shape {tuple(shape)}, got {tuple(t.shape)}")
    if t.device != device:
        raise ValueError(f"{name}: expected device {device}, got {t.device}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


def _L_of(states: torch.Tensor) -> int:
    if states.dim() != 2 or states.shape[1] % 2:
        raise ValueError(f"presentations must be (B, 2L), got {tuple(states.shape)}")
    L = states.shape[1] // 2
    if not 1 <= L <= _lib.MAX_L:
        raise ValueError(f"max_relator_length {L} outside [1, {_lib.MAX_L}]")
    return L


# relator lengths for which acx_step_lengths reads and writes only the live chunks (the kernels'
# compile-time tiles); at any other L it reads whole rows like acx_step
LIVE_TILE_L = (36, 128)
# where the lengths-carrying step measured faster than acx_step at any batch: L = 128 (config 5:
# 4.8e9 vs 3.8e9 env-steps/s per GPU over a horizon, round 4; with the reduced flags 7.5e9).  At
# L = 36 it wins only above the small-batch range (lengths_step_for)
LENGTHS_STEP_L = (128,)
# acx_step at a compile-time L = 36 tile with B <= this many envs runs the small-batch kernel
# (step_pair_kernel: two lanes per env, one per relator, so config 2's 65,536 envs are two waves
# per SIMD instead of one); csrc acx_kernels.hip SMALL_STEP_MAX_B
SMALL_STEP_MAX_B = 2 * 4 * 256 * 64


def lengths_step_for(B: int, L: int) -> bool:
    """whether VecACEnv.step (and bench.py's step headline) take the lengths-carrying step with
    reduced flags (acx_step_lengths_reduced): at L = 128, and at L = 36 above the small-batch
    range -- there a conjugation's unread relator makes it 5 % faster than acx_step at 2^20 envs
    (0.0683 vs 0.0719 ms, profiles/r06/r06k_ab_reduced_L36.json), while acx_step's two-lane kernel
    keeps the small batches"""
    return L in LENGTHS_STEP_L or (L == 36 and B > SMALL_STEP_MAX_B)


def step_kernel_name(B: int, L: int) -> str:
    """the kernel acx_step launches for B envs at max_relator_length L (bench lines, profiles)"""
    nw = 1 if L <= 16 else 2 if L <= 32 else 3 if L <= 48 else 4 if L <= 64 else 8
    lc = L if L in (36, 128) else 0
    if lc == 36 and B <= SMALL_STEP_MAX_B:
        return f"acx::step_pair_kernel<{nw},{lc},4>"
    return f"acx::step_kernel<{nw},{lc},4,false>"


def step(
    state_in: torch.Tensor,
    action: torch.Tensor,
    *,
    state_out: Optional[torch.Tensor] = None,
    reset_state: Optional[torch.Tensor] = None,
    step_count: Optional[torch.Tensor] = None,
    horizon: int = 0,
    cyclical: bool = True,
    reward: Optional[torch.Tensor] = None,
    done: Optional[torch.Tensor] = None,
    truncated: Optional[torch.Tensor] = None,
    lengths: Optional[torch.Tensor] = None,
    final_obs: Optional[torch.Tensor] = None,
    err: Optional[torch.Tensor] = None,
    err_count: Optional[torch.Tensor] = None,
    lengths_in: bool = False,
    reduced: Optional[torch.Tensor] = None,
) -> torch.Tensor:
    """acx_step: batched ACEnv.step / ACMove.  Returns state_out (in place if given as state_in).
    lengths_in: `lengths` already holds the rows' relator lengths (the previous call's output,
    or (L, L) for "unknown") and the step is in place -> acx_step_lengths, which reads and writes
    only the chunks inside the letters (ACMove's lengths in / lengths out, ac_moves.py:159,231).
    reduced (with lengths_in): (B,) uint8 per-row reduced flags, in/out (zeros for "unknown"; the
    previous call's output) -> acx_step_lengths_reduced, which also leaves the relator a
    conjugation does not touch unread when the row is known reduced (include/acx.h)."""
    lib = _lib.load()
    _need_gpu(state_in, "state_in")
    L = _L_of(state_in)
    B = state_in.shape[0]
    dev = state_in.device
    if state_out is None:
        state_out = torch.empty_like(state_in)
    _check(state_in, "state_in", _INT32, (B, 2 * L), dev)
    _check(state_out, "state_out", _INT32, (B, 2 * L), dev)
    _check(action, "action", _INT32, (B,), dev)
    _check(reset_state, "reset_state", _INT32, (B, 2 * L), dev)
    _check(step_count, "step_count", _INT32, (B,), dev)
    _check(reward, "reward", _INT32, (B,), dev)
    _check(done, "done", _UINT8, (B,), dev)
    _check(truncated, "truncated", _UINT8, (B,), dev)
    _check(lengths, "lengths", _INT32, (B, 2), dev)
    _check(final_obs, "final_obs", _INT32, (B, 2 * L), dev)
    _check(err, "err", _UINT8, (B,), dev)
    _check(err_count, "err_count", _INT32, (1,), dev)
    _check(reduced, "reduced", _UINT8, (B,), dev)
    if reduced is not None and not lengths_in:
        raise ValueError("reduced needs lengths_in (the lengths-carrying step)")
    if lengths_in:
        if lengths is None or state_out.data_ptr() != state_in.data_ptr():
            raise ValueError("lengths_in needs lengths and an in-place step (state_out is state_in)")
        if reduced is not None:
            st = lib.acx_step_lengths_reduced(
                _ptr(state_in), _ptr(action), _ptr(reset_state), _ptr(step_count), _ptr(reward), _ptr(done),
                _ptr(truncated), _ptr(lengths), _ptr(reduced), _ptr(final_obs), _ptr(err), _ptr(err_count),
                B, L, int(horizon), int(bool(cyclical)), _stream(dev),
            )
            _lib.check(st, "acx_step_lengths_reduced")
            return state_out
        st = lib.acx_step_lengths(
            _ptr(state_in), _ptr(action), _ptr(reset_state), _ptr(step_count), _ptr(reward), _ptr(done),
            _ptr(truncated), _ptr(lengths), _ptr(final_obs), _ptr(err), _ptr(err_count),
            B, L, int(horizon), int(bool(cyclical)), _stream(dev),
        )
        _lib.check(st, "acx_step_lengths")
        return state_out
    st = lib.acx_step(
        _ptr(state_in), _ptr(state_out), _ptr(action), _ptr(reset_state), _ptr(step_count), _ptr(reward),
        _ptr(done), _ptr(truncated), _ptr(lengths), _ptr(final_obs), _ptr(err), _ptr(err_count),
        B, L, int(horizon), int(bool(cyclical)), _stream(dev),
    )
    _lib.check(st, "acx_step")
    return state_out


def _check_rollout(state, reset_state, step_count, T, obs_traj, reward_traj, done_traj, trunc_traj, err, err_count):
    _need_gpu(state, "state")
    L = _L_of(state)
    B = state.shape[0]
    dev = state.device
    _check(state, "state", _INT32, (B, 2 * L), dev)
    _check(reset_state, "reset_state", _INT32, (B, 2 * L), dev)
    _check(step_count, "step_count", _INT32, (B,), dev)
    obs8 = obs_traj is not None and obs_traj.dtype == torch.int8
    _check(obs_traj, "obs_traj", torch.int8 if obs8 else _INT32, (T, B, 2 * L), dev)
    _check(reward_traj, "reward_traj", _INT32, (T, B), dev)
    _check(done_traj, "done_traj", _UINT8, (T, B), dev)
    _check(trunc_traj, "trunc_traj", _UINT8, (T, B), dev)
    _check(err, "err", _UINT8, (B,), dev)
    _check(err_count, "err_count", _INT32, (1,), dev)
    return L, B, dev, obs8


def packs_actions(T: int, obs_traj: Optional[torch.Tensor]) -> bool:
    """The move-id path ops.rollout / RolloutPlan take by default.  The rollout loads the ids of
    32 steps at a time when it writes an obs trajectory, so for T <= 32 every id load is issued
    before the first trajectory store and the int32 ids cost no store drain; the separate pack
    pass (a ~20-37 us launch at 2^20 envs) then costs more than the extra id bytes.  Measured
    in one process on the same buffers (tools/ab_pack.py, profiles/r03/r03v_ab_pack.json, 2^20
    envs, L = 36): int32 obs K = 20 1.350 vs 1.368 ms, K = 200 9.79 vs 9.63 ms (packed wins);
    int8 obs K = 20 0.475 vs 0.480, K = 200 3.750 vs 3.803 (int32 ids win)."""
    if obs_traj is None:
        return True
    return obs_traj.dtype != torch.int8 and T > 32


def rollout(
    state: torch.Tensor,
    actions: torch.Tensor,
    reset_state: torch.Tensor,
    step_count: torch.Tensor,
    *,
    horizon: int,
    cyclical: bool = True,
    obs_traj: Optional[torch.Tensor] = None,
    reward_traj: Optional[torch.Tensor] = None,
    done_traj: Optional[torch.Tensor] = None,
    trunc_traj: Optional[torch.Tensor] = None,
    err: Optional[torch.Tensor] = None,
    err_count: Optional[torch.Tensor] = None,
    pack_actions: Optional[bool] = None,
    packed_workspace: Optional[torch.Tensor] = None,
) -> None:
    """acx_rollout: T = actions.shape[0] fused env steps; state/step_count updated in place.

    pack_actions=True: acx_pack_actions + acx_rollout_packed -- one streaming pass packs the
    (T, B) int32 move ids 8 per word (0.5 B per env-step) into `packed_workspace`
    ((ceil(T/8), B) int32, allocated if not given), then the rollout reads those.
    pack_actions=False: the rollout reads the int32 ids itself (acx_rollout / acx_rollout_obs8).
    Identical results either way; None (default) picks by `packs_actions` (T, obs dtype).

    obs_traj may be int32 or int8 (T, B, 2L): int8 is the reference's observation dtype
    (ac_env.py:64-70) and goes to acx_rollout_obs8 (a quarter of the trajectory bytes)."""
    lib = _lib.load()
    T = actions.shape[0]
    L, B, dev, obs8 = _check_rollout(state, reset_state, step_count, T, obs_traj, reward_traj, done_traj, trunc_traj,
                                     err, err_count)
    _check(actions, "actions", _INT32, (T, B), dev)
    if pack_actions is None:
        pack_actions = packs_actions(T, obs_traj)
    if pack_actions and T > 0 and B > 0:
        words = (T + 7) // 8
        if packed_workspace is None:
            packed_workspace = torch.empty((words, B), dtype=_INT32, device=dev)
        elif (packed_workspace.dtype != _INT32 or packed_workspace.device != dev or not packed_workspace.is_contiguous()
              or packed_workspace.numel() < words * B):
            raise ValueError(f"packed_workspace must be a contiguous int32 tensor of >= {words * B} elements on {dev}")
        st = lib.acx_pack_actions(_ptr(actions), _ptr(packed_workspace), T, B, _stream(dev))
        _lib.check(st, "acx_pack_actions")
        if obs8:
            st = lib.acx_rollout_obs8(
                _ptr(state), None, _ptr(packed_workspace), _ptr(reset_state), _ptr(step_count), _ptr(obs_traj),
                _ptr(reward_traj), _ptr(done_traj), _ptr(trunc_traj), _ptr(err), _ptr(err_count), T, B, L,
                int(horizon), int(bool(cyclical)), _stream(dev),
            )
            _lib.check(st, "acx_rollout_obs8")
            return
        st = lib.acx_rollout_packed(
            _ptr(state), _ptr(packed_workspace), _ptr(reset_state), _ptr(step_count), _ptr(obs_traj),
            _ptr(reward_traj), _ptr(done_traj), _ptr(trunc_traj), _ptr(err), _ptr(err_count), T, B, L, int(horizon),
            int(bool(cyclical)), _stream(dev),
        )
        _lib.check(st, "acx_rollout_packed")
        return
    if obs8:
        st = lib.acx_rollout_obs8(
            _ptr(state), _ptr(actions), None, _ptr(reset_state), _ptr(step_count), _ptr(obs_traj), _ptr(reward_traj),
            _ptr(done_traj), _ptr(trunc_traj), _ptr(err), _ptr(err_count), T, B, L, int(horizon),
            int(bool(cyclical)), _stream(dev),
        )
        _lib.check(st, "acx_rollout_obs8")
        return
    st = lib.acx_rollout(
        _ptr(state), _ptr(actions), _ptr(reset_state), _ptr(step_count), _ptr(obs_traj), _ptr(reward_traj),
        _ptr(done_traj), _ptr(trunc_traj), _ptr(err), _ptr(err_count), T, B, L, int(horizon),
        int(bool(cyclical)), _stream(dev),
    )
    _lib.check(st, "acx_rollout")


class RolloutPlan:
    """ops.rollout over buffers fixed once: the argument checks, the pointer lookups, the
    move-id path (`packs_actions`, or `pack_actions`) and the packed-move workspace are settled
    here, so each call only checks the (T, B) actions tensor and issues the launches
    (acx_pack_actions + acx_rollout_packed / acx_rollout_obs8, or acx_rollout /
    acx_rollout_obs8 on the int32 ids) on the current stream.  This is what a PPO loop that
    reuses its rollout storage every update calls; results are identical to ops.rollout with the
    same arguments.  The plan keeps references to its tensors; their storage must not be
    resized or replaced."""

    def __init__(
        self,
        state: torch.Tensor,
        reset_state: torch.Tensor,
        step_count: torch.Tensor,
        *,
        T: int,
        horizon: int,
        cyclical: bool = True,
        obs_traj: Optional[torch.Tensor] = None,
        reward_traj: Optional[torch.Tensor] = None,
        done_traj: Optional[torch.Tensor] = None,
        trunc_traj: Optional[torch.Tensor] = None,
        err: Optional[torch.Tensor] = None,
        err_count: Optional[torch.Tensor] = None,
        pack_actions: Optional[bool] = None,
    ):
        lib = _lib.load()
        T = int(T)
        if T < 0:
            raise ValueError(f"T must be >= 0, got {T}")
        L, B, dev, obs8 = _check_rollout(state, reset_state, step_count, T, obs_traj, reward_traj, done_traj,
                                         trunc_traj, err, err_count)
        self.T, self.B, self.L, self.device = T, B, L, dev
        self.packs = packs_actions(T, obs_traj) if pack_actions is None else bool(pack_actions)
        self._ashape = torch.Size((T, B))
        self._keep = (state, reset_state, step_count, obs_traj, reward_traj, done_traj, trunc_traj, err, err_count)
        tail = (_ptr(reset_state), _ptr(step_count), _ptr(obs_traj), _ptr(reward_traj), _ptr(done_traj),
                _ptr(trunc_traj), _ptr(err), _ptr(err_count), T, B, L, int(horizon), int(bool(cyclical)))
        self._head = (_ptr(state),)
        if self.packs:
            self._ws = torch.empty(((T + 7) // 8, B), dtype=_INT32, device=dev)
            self._wsp = self._ws.data_ptr()
            self._pack = lib.acx_pack_actions
            if obs8:
                self._fn, self._name = lib.acx_rollout_obs8, "acx_rollout_obs8"
                self._args = (_ptr(state), None, self._wsp) + tail
            else:
                self._fn, self._name = lib.acx_rollout_packed, "acx_rollout_packed"
                self._args = (_ptr(state), self._wsp) + tail
        elif obs8:  # the action pointer goes in per call: (state, actions, packed=None, ...)
            self._fn, self._name, self._tail = lib.acx_rollout_obs8, "acx_rollout_obs8", (None,) + tail
        else:
            self._fn, self._name, self._tail = lib.acx_rollout, "acx_rollout", tail

    def __call__(self, actions: torch.Tensor) -> None:
        """T fused env steps with `actions` ((T, B) int32, contiguous, on the plan's device)."""
        if (actions.shape != self._ashape or actions.dtype != _INT32 or actions.device != self.device
                or not actions.is_contiguous()):
            raise ValueError(f"actions must be a contiguous int32 tensor of shape {tuple(self._ashape)} on "
                             f"{self.device}, got {actions.dtype} {tuple(actions.shape)} on {actions.device}")
        if self.T == 0 or self.B == 0:
            return
        s = _stream(self.device)
        if self.packs:
            _lib.check(self._pack(actions.data_ptr(), self._wsp, self.T, self.B, s), "acx_pack_actions")
            _lib.check(self._fn(*self._args, s), self._name)
        else:
            _lib.check(self._fn(*self._head, actions.data_ptr(), *self._tail, s), self._name)


class StepPlan:
    """ops.step with its arguments checked and resolved once: a loop that steps the same buffers
    every call (a small batch stepped many times: BASELINE configs[1]) pays one ctypes call per
    step instead of ops.step's per-call checks, and that call is acx_step_plan_launch's three
    arguments (include/acx.h) -- at 65,536 envs the kernel is ~6.5 us, and the host, not the GPU,
    set the eager rate.  Same kernels and results as ops.step with the same arguments
    (lengths_in=True: acx_step_lengths; with reduced: acx_step_lengths_reduced).  The plan keeps
    references to its tensors; their storage must not be resized or replaced."""

    def __init__(
        self,
        state_in: torch.Tensor,
        *,
        state_out: Optional[torch.Tensor] = None,
        reset_state: Optional[torch.Tensor] = None,
        step_count: Optional[torch.Tensor] = None,
        horizon: int = 0,
        cyclical: bool = True,
        reward: Optional[torch.Tensor] = None,
        done: Optional[torch.Tensor] = None,
        truncated: Optional[torch.Tensor] = None,
        lengths: Optional[torch.Tensor] = None,
        final_obs: Optional[torch.Tensor] = None,
        err: Optional[torch.Tensor] = None,
        err_count: Optional[torch.Tensor] = None,
        lengths_in: bool = False,
        reduced: Optional[torch.Tensor] = None,
    ):
        lib = _lib.load()
        _need_gpu(state_in, "state_in")
        L = _L_of(state_in)
        B = state_in.shape[0]
        dev = state_in.device
        if state_out is None:
            state_out = state_in
        rows, per_env = (B, 2 * L), (B,)
        for t, name, dt, shape in (
                (state_in, "state_in", _INT32, rows), (state_out, "state_out", _INT32, rows),
                (reset_state, "reset_state", _INT32, rows), (step_count, "step_count", _INT32, per_env),
                (reward, "reward", _INT32, per_env), (done, "done", _UINT8, per_env),
                (truncated, "truncated", _UINT8, per_env), (lengths, "lengths", _INT32, (B, 2)),
                (final_obs, "final_obs", _INT32, rows), (err, "err", _UINT8, per_env),
                (err_count, "err_count", _INT32, (1,)), (reduced, "reduced", _UINT8, per_env)):
            _check(t, name, dt, shape, dev)
        if reduced is not None and not lengths_in:
            raise ValueError("reduced needs lengths_in (the lengths-carrying step)")
        self.B, self.L, self.device, self.state_out = B, L, dev, state_out
        self._didx = dev.index if dev.index is not None else torch.cuda.current_device()
        self._ashape = torch.Size((B,))
        self._keep = (state_in, state_out, reset_state, step_count, reward, done, truncated, lengths, final_obs, err,
                      err_count, reduced)
        if lengths_in and (lengths is None or state_out.data_ptr() != state_in.data_ptr()):
            raise ValueError("lengths_in needs lengths and an in-place step (state_out is state_in)")
        # the launch is acx_step_plan_launch(plan, action, stream): three ctypes arguments instead of
        # the entry's seventeen (~2.4 us of host time per call saved, as much as a third of the
        # kernel at 65,536 envs)
        if not lengths_in:
            kind, self._name = 0, "acx_step"
        elif reduced is None:
            kind, self._name = 1, "acx_step_lengths"
        else:
            kind, self._name = 2, "acx_step_lengths_reduced"
        self._lib = lib
        self._plan = lib.acx_step_plan_create(
            kind, _ptr(state_in), _ptr(state_out), _ptr(reset_state), _ptr(step_count), _ptr(reward), _ptr(done),
            _ptr(truncated), _ptr(lengths), _ptr(reduced), _ptr(final_obs), _ptr(err), _ptr(err_count), B, L,
            int(horizon), int(bool(cyclical)))
        if not self._plan:
            _lib.check(_lib.E_ARG, f"acx_step_plan_create ({self._name})")
        self._launch = lib.acx_step_plan_launch

    def __del__(self):
        plan, self._plan = getattr(self, "_plan", None), None
        if plan:
            self._lib.acx_step_plan_destroy(plan)

    def __call__(self, action: torch.Tensor) -> torch.Tensor:
        """One env step with `action` ((B,) int32, contiguous, on the plan's device)."""
        if (action.shape != self._ashape or action.dtype != _INT32 or action.get_device() != self._didx
                or not action.is_contiguous()):
            raise ValueError(f"action must be a contiguous int32 tensor of shape {tuple(self._ashape)} on "
                             f"{self.device}, got {action.dtype} {tuple(action.shape)} on {action.device}")
        if self.B:
            rc = self._launch(self._plan, action.data_ptr(), _stream(self.device))
            if rc:
                _lib.check(rc, self._name)
        return self.state_out


def expand12(
    parents: torch.Tensor,
    *,
    cyclical: bool = False,
    children: bool = True,
    lengths: bool = True,
    keys: bool = False,
    err: bool = True,
    out: Optional[dict] = None,
):
    """acx_expand12: all 12 ACMove children of every parent.

    Returns a dict with (as requested) "children" (N,12,2L) int32, "lengths" (N,12,2) int32,
    "keys" (N,12,KW) int64 (packed states), "err" (N,12) uint8.  Pass `out` (a dict of
    preallocated tensors with those names) to reuse buffers.
    """
    lib = _lib.load()
    _need_gpu(parents, "parents")
    L = _L_of(parents)
    N = parents.shape[0]
    dev = parents.device
    kw = _lib.key_words(L)
    _check(parents, "parents", _INT32, (N, 2 * L), dev)
    res = {}
    spec = {
        "children": (children, _INT32, (N, 12, 2 * L)),
        "lengths": (lengths, _INT32, (N, 12, 2)),
        "keys": (keys, torch.int64, (N, 12, kw)),
        "err": (err, _UINT8, (N, 12)),
    }
    for name, (want, dt, shape) in spec.items():
        if not want:
            continue
        t = out.get(name) if out else None
        if t is None:
            t = torch.empty(shape, dtype=dt, device=dev)
        else:
            t = t[: shape[0]] if t.shape[0] != shape[0] else t
            _check(t, name, dt, shape, dev)
        res[name] = t
    st = lib.acx_expand12(
        _ptr(parents), _ptr(res.get("children")), _ptr(res.get("lengths")), _ptr(res.get("keys")),
        _ptr(res.get("err")), None, N, L, int(bool(cyclical)), _stream(dev),
    )
    _lib.check(st, "acx_expand12")
    return res


def canonicalize(states: torch.Tensor, *, cyclical: bool = True, out: Optional[torch.Tensor] = None):
    """acx_canonicalize: simplify_presentation over a batch -> (states, lengths (B,2), err (B,))."""
    lib = _lib.load()
    _need_gpu(states, "states")
    L = _L_of(states)
    B = states.shape[0]
    dev = states.device
    _check(states, "states", _INT32, (B, 2 * L), dev)
    if out is None:
        out = torch.empty_like(states)
    lens = torch.empty((B, 2), dtype=_INT32, device=dev)
    err = torch.empty((B,), dtype=_UINT8, device=dev)
    st = lib.acx_canonicalize(_ptr(states), _ptr(out), _ptr(lens), _ptr(err), None, B, L, int(bool(cyclical)),
                              _stream(dev))
    _lib.check(st, "acx_canonicalize")
    return out, lens, err


def unpack_keys(keys: torch.Tensor, L: int, *, out: Optional[torch.Tensor] = None, lengths: bool = False):
    """acx_unpack_keys: packed keys (M, KW) int64 -> presentations (M, 2L) int32 (+ lengths)."""
    lib = _lib.load()
    _need_gpu(keys, "keys")
    kw = _lib.key_words(L)
    keys = keys.reshape(-1, kw)
    M = keys.shape[0]
    dev = keys.device
    _check(keys, "keys", torch.int64, (M, kw), dev)
    if out is None:
        out = torch.empty((M, 2 * L), dtype=_INT32, device=dev)
    _check(out, "out", _INT32, (M, 2 * L), dev)
    lens = torch.empty((M, 2), dtype=_INT32, device=dev) if lengths else None
    st = lib.acx_unpack_keys(_ptr(keys), _ptr(out), _ptr(lens), M, int(L), _stream(dev))
    _lib.check(st, "acx_unpack_keys")
    return (out, lens) if lengths else out


def _states_or_keys(states, keys, L):
    if (states is None) == (keys is None):
        raise ValueError("pass exactly one of states= or keys=")
    if states is not None:
        _need_gpu(states, "states")
        L = _L_of(states)
        M = states.shape[0]
        _check(states, "states", _INT32, (M, 2 * L), states.device)
        return states, None, L, M, states.device
    if L is None:
        raise ValueError("keys= needs L")
    _need_gpu(keys, "keys")
    kw = _lib.key_words(L)
    keys = keys.reshape(-1, kw)
    M = keys.shape[0]
    _check(keys, "keys", torch.int64, (M, kw), keys.device)
    return None, keys, int(L), M, keys.device


def features(*, states: Optional[torch.Tensor] = None, keys: Optional[torch.Tensor] = None, L: Optional[int] = None,
             mean: Optional[torch.Tensor] = None, std: Optional[torch.Tensor] = None,
             out: Optional[torch.Tensor] = None):
    """acx_features: the 14 features of value_search/feature_extraction.py:11-91 per presentation
    ((M,2L) int32 states, or packed keys with L) -> (M,14) float32; normalised (f - mean)/std
    when mean and std (14 float32 each) are given, as value_guided_search.py:49-66."""
    lib = _lib.load()
    states, keys, L, M, dev = _states_or_keys(states, keys, L)
    if (mean is None) != (std is None):
        raise ValueError("pass both mean and std, or neither")
    for name, t in (("mean", mean), ("std", std)):
        _check(t, name, torch.float32, (14,), dev)
    if out is None:
        out = torch.empty((M, 14), dtype=torch.float32, device=dev)
    _check(out, "out", torch.float32, (M, 14), dev)
    st = lib.acx_features(_ptr(states), _ptr(keys), _ptr(mean), _ptr(std), _ptr(out), M, L, _stream(dev))
    _lib.check(st, "acx_features")
    return out


def token_ids(*, states: Optional[torch.Tensor] = None, keys: Optional[torch.Tensor] = None, L: Optional[int] = None,
              max_state_dim: Optional[int] = None, out: Optional[torch.Tensor] = None):
    """acx_token_ids: SequenceValueNet input (value_guided_search.py:68-84): letter + 2 as int64,
    padded with 2 to max_state_dim (default 2L) -> (M, max_state_dim) int64."""
    lib = _lib.load()
    states, keys, L, M, dev = _states_or_keys(states, keys, L)
    D = 2 * L if max_state_dim is None else int(max_state_dim)
    if D < 2 * L:
        raise ValueError(f"max_state_dim {D} < 2L = {2 * L}")
    if out is None:
        out = torch.empty((M, D), dtype=torch.int64, device=dev)
    _check(out, "out", torch.int64, (M, D), dev)
    st = lib.acx_token_ids(_ptr(states), _ptr(keys), _ptr(out), M, L, D, _stream(dev))
    _lib.check(st, "acx_token_ids")
    return out


# ---------------------------------------------------------------------------------------------
# exact word functions on arbitrary int32 letters (csrc/acx_words.hip)
# ---------------------------------------------------------------------------------------------
def _word_setup(states: torch.Tensor, name: str):
    _need_gpu(states, name)
    if states.dim() != 2 or states.shape[1] % 2 or states.shape[1] == 0:
        raise ValueError(f"{name} must be (B, 2L), got {tuple(states.shape)}")
    if states.dtype != _INT32 or not states.is_contiguous():
        raise TypeError(f"{name} must be a contiguous int32 tensor")
    return states.shape[0], states.shape[1] // 2, states.device


def word_move(states: torch.Tensor, action: torch.Tensor, *, cyclical: bool = True):
    """acx_word_move: ACMove (ac_moves.py:159-231) on arbitrary letters, one move id per row.
    Returns (out, lengths (B,2), done (B) strict triviality, err (B) ACX_ERR_* codes)."""
    lib = _lib.load()
    B, L, dev = _word_setup(states, "states")
    _check(action, "action", _INT32, (B,), dev)
    out = torch.empty_like(states)
    lens = torch.empty((B, 2), dtype=_INT32, device=dev)
    done = torch.empty(B, dtype=_UINT8, device=dev)
    err = torch.empty(B, dtype=_UINT8, device=dev)
    st = lib.acx_word_move(_ptr(states), _ptr(out), _ptr(action), _ptr(lens), _ptr(done), _ptr(err), None, B, L,
                           int(bool(cyclical)), _stream(dev))
    _lib.check(st, "acx_word_move")
    return out, lens, done, err


def concatenate(states: torch.Tensor, i: int, j: int, sign: int, lengths: Optional[torch.Tensor] = None):
    """acx_concatenate: concatenate_relators (ac_moves.py:4-76) over a batch, r_i <- r_i r_j^sign,
    no reduction.  Returns (out, lengths_out)."""
    lib = _lib.load()
    B, L, dev = _word_setup(states, "states")
    _check(lengths, "lengths", _INT32, (B, 2), dev)
    out = torch.empty_like(states)
    lo = torch.empty((B, 2), dtype=_INT32, device=dev)
    st = lib.acx_concatenate(_ptr(states), _ptr(out), _ptr(lengths), _ptr(lo), B, L, int(i), int(j), int(sign),
                             _stream(dev))
    _lib.check(st, "acx_concatenate")
    return out, lo


def conjugate(states: torch.Tensor, i: int, j: int, sign: int, lengths: Optional[torch.Tensor] = None):
    """acx_conjugate: conjugate (ac_moves.py:79-156) over a batch, r_i <- x_j^sign r_i x_j^-sign,
    no reduction.  Returns (out, lengths_out, err) -- err 2 where the reference raises IndexError."""
    lib = _lib.load()
    B, L, dev = _word_setup(states, "states")
    _check(lengths, "lengths", _INT32, (B, 2), dev)
    out = torch.empty_like(states)
    lo = torch.empty((B, 2), dtype=_INT32, device=dev)
    err = torch.empty(B, dtype=_UINT8, device=dev)
    st = lib.acx_conjugate(_ptr(states), _ptr(out), _ptr(lengths), _ptr(lo), _ptr(err), None, B, L, int(i), int(j),
                           int(sign), _stream(dev))
    _lib.check(st, "acx_conjugate")
    return out, lo, err


def word_simplify_presentation(states: torch.Tensor, *, cyclical: bool = True):
    """acx_word_simplify_presentation: simplify_presentation (utils.py:246-283) on arbitrary
    letters.  Returns (out, lengths, err)."""
    lib = _lib.load()
    B, L, dev = _word_setup(states, "states")
    out = torch.empty_like(states)
    lo = torch.empty((B, 2), dtype=_INT32, device=dev)
    err = torch.empty(B, dtype=_UINT8, device=dev)
    st = lib.acx_word_simplify_presentation(_ptr(states), _ptr(out), _ptr(lo), _ptr(err), None, B, L,
                                            int(bool(cyclical)), _stream(dev))
    _lib.check(st, "acx_word_simplify_presentation")
    return out, lo, err


def word_simplify_relator(relators: torch.Tensor, max_relator_length: int, *, cyclical: bool = False,
                          padded: bool = True):
    """acx_word_simplify_relator: simplify_relator (utils.py:178-243) on (B, m) relator arrays.
    Returns (out (B, max(m, L)), out_len (B), n (B), err (B)): row b's returned array is
    out[b, :out_len[b]]."""
    lib = _lib.load()
    _need_gpu(relators, "relators")
    if relators.dim() != 2 or relators.dtype != _INT32 or not relators.is_contiguous():
        raise TypeError("relators must be a contiguous (B, m) int32 tensor")
    B, m = relators.shape
    L = int(max_relator_length)
    dev = relators.device
    out = torch.empty((B, max(m, L)), dtype=_INT32, device=dev)
    ol = torch.empty(B, dtype=_INT32, device=dev)
    n = torch.zeros(B, dtype=_INT32, device=dev)
    err = torch.empty(B, dtype=_UINT8, device=dev)
    st = lib.acx_word_simplify_relator(_ptr(relators), m, _ptr(out), _ptr(ol), _ptr(n), _ptr(err), None, B, L,
                                       int(bool(cyclical)), int(bool(padded)), _stream(dev))
    _lib.check(st, "acx_word_simplify_relator")
    return out, ol, n, err
