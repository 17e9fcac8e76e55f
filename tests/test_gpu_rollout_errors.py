"""GPU: the error contract of the fused rollout equals T repeated acx_step calls.

The reference raises inside ACEnv.step before `count_steps += 1` (ac_env.py:93-103), so the
batched API's contract (include/acx.h) is: an env whose move fails (err 1 a relator emptied,
utils.py:264-266; err 4 a move id outside [0,12), ac_moves.py:188-190) keeps its state and
step count for that step (done = truncated = 0, reward = -(n0+n1)); an env whose row is outside
the packed domain (err 3: a letter outside {-2..2} or a zero inside a relator -- its input row,
or a starting row an autoreset loaded, which is then held as that row with count 0, as the
reference's reset takes any row, ac_env.py:113-129) never moves and never counts.

Every stream here mixes all of those with ordinary moves, desynchronised autoresets (a few
lanes or a whole wave at once) and every tile type (L = 36 FastTile, 128 CodeTile, 17 generic).
The rollout (int32 or int8 observations, packed or int32 ids) is compared step by step with T
in-place acx_step calls and with `_model_step` below: the same contract over the C oracle's
ACMove (oracle/acx_oracle.c, pinned to the reference's fixtures) for the rows that move.
"""
import os

import numpy as np
import pytest
import torch

from conftest import env_step_contract

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


def _model_step(st, a, cnt, resets, L, H):
    return env_step_contract(st, a, cnt, resets, L, H, True)


def _starts(L, B, seed):
    import acx
    ms = np.load(os.path.join(os.path.dirname(acx.__file__), "data", "all_presentations.npy"))
    rng = np.random.default_rng(seed)
    out = np.zeros((B, 2 * L), np.int32)
    for i in range(B):
        p = ms[rng.integers(len(ms))]
        a, b = p[:18][p[:18] != 0][:L], p[18:][p[18:] != 0][:L]
        out[i, :len(a)] = a
        out[i, L:L + len(b)] = b
    return out


def _error_stream(L, B, T, H, seed):
    """starting rows, reset rows, initial counts and (T, B) ids with every error kind"""
    rng = np.random.default_rng(seed)
    st = _starts(L, B, seed)
    # r0 == r1: moves 1 (r0 <- r0 r1^-1) and 2 (r1 <- r1 r0^-1) empty a relator (err 1)
    eq = rng.choice(B, size=B // 6, replace=False)
    st[eq, L:] = st[eq, :L]
    # an unreduced r0 = y^-1 y: the first move's reduction empties it (no error: the reference
    # checks validity before reducing, utils.py:264-266); conjugating it then raises (err 2)
    emp = rng.choice(np.setdiff1d(np.arange(B), eq), size=B // 12, replace=False)
    st[emp, :L] = 0
    st[emp, 0], st[emp, 1] = -2, 2
    resets = st.copy()
    # out-of-domain input rows (err 3 from step 0): a letter 3, a zero inside r1, a letter 300
    bad_in = rng.choice(np.setdiff1d(np.arange(B), np.concatenate([eq, emp])), size=9, replace=False)
    st[bad_in[:3], 0] = 3
    st[bad_in[3:6], L + 1] = 0
    st[bad_in[3:6], L + 2] = 1
    st[bad_in[6:], 1] = 300
    # out-of-domain starting rows (err 3 at the env's first autoreset)
    bad_rs = rng.choice(np.setdiff1d(np.arange(B), np.concatenate([eq, emp, bad_in])), size=7, replace=False)
    resets[bad_rs[:3], L] = -5
    resets[bad_rs[3:], 2] = 0
    resets[bad_rs[3:], 3] = -2
    acts = rng.integers(0, 12, size=(T, B)).astype(np.int32)
    # r0 == r1 rows: move 1 / 2 often, so emptying concatenations happen (also after resets)
    hot = rng.random((T, B)) < 0.4
    acts[:, eq] = np.where(hot[:, eq], rng.choice(np.array([1, 2], np.int32), size=(T, len(eq))), acts[:, eq])
    bad_id = rng.random((T, B)) < 0.03
    acts[bad_id] = rng.choice(np.array([12, 15, -1, 1 << 20], np.int32), size=int(bad_id.sum()))
    count0 = (np.arange(B) % H).astype(np.int32)
    # one wave in sync (a whole-tile reload when it truncates)
    count0[64:128] = 0
    return st, resets, count0, acts, eq, bad_in, bad_rs


def _rollout(st, resets, count0, acts, L, H, pack, obs_dtype):
    from acx import ops
    T, B = acts.shape
    s = torch.as_tensor(st).to(DEV)
    rs = torch.as_tensor(resets).to(DEV)
    cnt = torch.as_tensor(count0).to(DEV)
    obs = torch.full((T, B, 2 * L), -7, dtype=obs_dtype, device=DEV)
    rew = torch.zeros((T, B), dtype=torch.int32, device=DEV)
    dn = torch.zeros((T, B), dtype=torch.uint8, device=DEV)
    tr = torch.zeros((T, B), dtype=torch.uint8, device=DEV)
    err = torch.zeros(B, dtype=torch.uint8, device=DEV)
    ec = torch.zeros(1, dtype=torch.int32, device=DEV)
    ops.rollout(s, torch.as_tensor(acts).to(DEV), rs, cnt, horizon=H, cyclical=True, obs_traj=obs, reward_traj=rew,
                done_traj=dn, trunc_traj=tr, err=err, err_count=ec, pack_actions=pack)
    return [x.cpu().numpy() for x in (s, cnt, obs, rew, dn, tr, err, ec)]


def _repeated_steps(st, resets, count0, acts, L, H, in_place=True):
    from acx import ops
    T, B = acts.shape
    s = torch.as_tensor(st).to(DEV)
    rs = torch.as_tensor(resets).to(DEV)
    cnt = torch.as_tensor(count0).to(DEV)
    rew = torch.zeros(B, dtype=torch.int32, device=DEV)
    dn = torch.zeros(B, dtype=torch.uint8, device=DEV)
    tr = torch.zeros(B, dtype=torch.uint8, device=DEV)
    lens = torch.zeros((B, 2), dtype=torch.int32, device=DEV)
    err = torch.zeros(B, dtype=torch.uint8, device=DEV)
    out = []
    for t in range(T):
        dst = s if in_place else torch.empty_like(s)
        ops.step(s, torch.as_tensor(acts[t]).to(DEV), state_out=dst, reset_state=rs, step_count=cnt, horizon=H,
                 cyclical=True, reward=rew, done=dn, truncated=tr, lengths=lens, err=err)
        s = dst
        out.append([x.cpu().numpy().copy() for x in (s, cnt, rew, dn, tr, err, lens)])
    return out


@pytest.mark.parametrize("L", [36, 128, 17])
@pytest.mark.parametrize("in_place", [True, False])
def test_step_api_error_contract_vs_model(L, in_place):
    """acx_step, in place (dirty-relator write-back) and out of place (fallback rows), against the
    contract model step by step: states, counts, rewards, done, truncated, errors, lengths."""
    B, T, H = 64 * 11 + 21, 26, 6
    st, resets, count0, acts, eq, bad_in, bad_rs = _error_stream(L, B, T, H, seed=L + 1)
    steps = _repeated_steps(st, resets, count0, acts, L, H, in_place=in_place)
    m_st, m_cnt = st.copy(), count0.copy()
    seen = np.zeros(5, bool)
    for t in range(T):
        r, d, trn, e = _model_step(m_st, acts[t], m_cnt, resets, L, H)
        g_st, g_cnt, g_rew, g_dn, g_tr, g_err, g_len = steps[t]
        assert np.array_equal(g_st, m_st), t
        assert np.array_equal(g_cnt, m_cnt), t
        assert np.array_equal(g_rew, r) and np.array_equal(g_dn, d) and np.array_equal(g_tr, trn), t
        assert np.array_equal(g_err, e), t
        n = np.stack([(m_st[:, :L] != 0).sum(1), (m_st[:, L:] != 0).sum(1)], 1)
        assert np.array_equal(g_len, n), t
        for k in (1, 2, 3, 4):
            seen[k] |= (e == k).any()
        seen[0] |= bool((d | trn).any())
    assert seen.all(), seen  # every error kind and resets occurred
    assert (steps[-1][0][bad_rs] == resets[bad_rs]).all()  # held as the out-of-domain starting row


@pytest.mark.parametrize("L", [36, 128, 17])
@pytest.mark.parametrize("pack", [True, False])
@pytest.mark.parametrize("obs_dtype", [torch.int32, torch.int8])
def test_rollout_with_errors_equals_repeated_step(L, pack, obs_dtype):
    """The fused rollout over a stream with every error kind = T repeated acx_step calls = the
    contract model (oracle ACMove on the rows that move): per-step observations (exact values of
    out-of-domain rows, int8-wrapped for the int8 trajectory), rewards, done, truncated; the final
    states and counts; err = the first error of each env; err_count."""
    B, T, H = 64 * 11 + 21, 26, 6
    st, resets, count0, acts, eq, bad_in, bad_rs = _error_stream(L, B, T, H, seed=L + 1)
    g = _rollout(st, resets, count0, acts, L, H, pack, obs_dtype)
    steps = _repeated_steps(st, resets, count0, acts, L, H)
    m_st, m_cnt = st.copy(), count0.copy()
    first_err = np.zeros(B, np.uint8)
    for t in range(T):
        r, d, trn, e = _model_step(m_st, acts[t], m_cnt, resets, L, H)
        first_err = np.where(first_err == 0, e, first_err)
        s_st, s_cnt, s_rew, s_dn, s_tr, s_err, _ = steps[t]
        assert np.array_equal(s_st, m_st) and np.array_equal(s_cnt, m_cnt), t
        want_obs = m_st.astype(np.int8) if obs_dtype == torch.int8 else m_st
        assert np.array_equal(g[2][t], want_obs), t
        assert np.array_equal(g[3][t], r) and np.array_equal(g[3][t], s_rew), t
        assert np.array_equal(g[4][t], d) and np.array_equal(g[4][t], s_dn), t
        assert np.array_equal(g[5][t], trn) and np.array_equal(g[5][t], s_tr), t
    assert np.array_equal(g[0], m_st) and np.array_equal(g[1], m_cnt)
    assert np.array_equal(g[6], first_err)
    assert int(g[7][0]) == int((first_err != 0).sum())
    assert (first_err[eq] == 1).sum() > 0 and (first_err == 4).any()
    assert (first_err[bad_in] == 3).all() and (first_err[bad_rs] != 0).all()  # a bad id may come first
    assert np.array_equal(g[0][bad_in], st[bad_in]) and np.array_equal(g[1][bad_in], count0[bad_in])
    assert np.array_equal(g[0][bad_rs], resets[bad_rs]) and (g[1][bad_rs] == 0).all()
