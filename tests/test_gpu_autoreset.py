"""GPU: gymnasium >= 1.0's NEXT_STEP autoreset (VecACEnv(autoreset_mode="next_step") ->
acx_step_next) against a host model built on the oracle's ACEnv.step without autoreset
(oracle/acx_oracle.c): the step that ends an episode returns the terminal state; the env's next
step resets it instead of moving (action ignored, reward 0, done = truncated = 0, count 0).
Parity unpinned upstream (gymnasium is an un-vendored dependency); the per-step
semantics are the oracle's, which is pinned to the reference's fixtures."""
import numpy as np
import pytest
import torch

from conftest import REPO  # noqa: F401

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


def _starts(L, B):
    from bench import ms_starts
    st = ms_starts(L, B)
    triv = np.zeros((8, 2 * L), np.int32)
    for r, (a0, a1) in enumerate([(1, 2), (1, -2), (-1, 2), (-1, -2), (2, 1), (2, -1), (-2, 1), (-2, -1)]):
        triv[r, 0], triv[r, L] = a0, a1
    st[::3] = triv[np.arange(B)[::3] % 8]  # a third start trivial: episodes end often
    return st


@pytest.mark.parametrize("L,record", [(36, False), (36, True), (128, False), (18, True)])
def test_next_step_autoreset_matches_oracle_model(L, record):
    from acx.envs.ac_env import VecACEnv
    from oracle import oracle as O
    B, H, T = 3000, 7, 30
    starts = _starts(L, B)
    env = VecACEnv(starts, horizon_length=H, device=DEV, record_actions=record, info_format="actions",
                   autoreset_mode="next_step")
    rng = np.random.default_rng(L)
    state = starts.copy()
    count = np.zeros(B, np.int32)
    pending = np.zeros(B, bool)
    hist = [[] for _ in range(B)]
    n_done = n_trunc = n_reset = 0
    for t in range(T):
        a = rng.integers(0, 12, size=B).astype(np.int32)
        obs, rew, dn, tr, info = env.step(torch.as_tensor(a, device=DEV))
        # model: pending envs reset, the others take the oracle's step (no autoreset)
        m_rew = np.zeros(B, np.int32)
        m_dn = np.zeros(B, np.uint8)
        m_tr = np.zeros(B, np.uint8)
        go = ~pending
        idx = np.nonzero(go)[0]
        sub = np.ascontiguousarray(state[idx])
        cnt = np.ascontiguousarray(count[idx])
        r, d, tt, err, _, _ = O.env_step(sub, a[idx], L, H, cnt)
        assert not err.any()
        state[idx], count[idx] = sub, cnt
        m_rew[idx], m_dn[idx], m_tr[idx] = r, d, tt
        for k, i in enumerate(idx):
            hist[i].append(int(a[i]))
        rs = np.nonzero(pending)[0]
        state[rs], count[rs] = starts[rs], 0
        for i in rs:
            hist[i] = []
        n_reset += len(rs)
        assert np.array_equal(obs.cpu().numpy(), state), t
        assert np.array_equal(rew.cpu().numpy(), m_rew), t
        assert np.array_equal(dn.cpu().numpy(), m_dn), t
        assert np.array_equal(tr.cpu().numpy(), m_tr), t
        assert np.array_equal(env.step_count.cpu().numpy(), count), t
        if record:
            solved = np.nonzero(m_dn)[0]
            if len(solved):
                assert info["_actions"].tolist() == m_dn.astype(bool).tolist()
                for i in solved:
                    assert list(info["actions"][i]) == hist[i], (t, i)
        n_done += int(m_dn.sum())
        n_trunc += int(m_tr.sum())
        pending = (m_dn | m_tr).astype(bool)
    assert n_done > 50 and n_trunc > 50 and n_reset > 100  # every path exercised
    assert int(env.err_count.item()) == 0


def test_next_step_mode_rejects_final_info_layout():
    from acx.envs.ac_env import VecACEnv
    with pytest.raises(ValueError):
        VecACEnv(_starts(36, 64), device=DEV, record_actions=True, info_format="final_info",
                 autoreset_mode="next_step")
    with pytest.raises(ValueError):
        VecACEnv(_starts(36, 64), device=DEV, autoreset_mode="bogus")


def test_rollout_refuses_per_env_state_it_cannot_keep():
    """The fused rollout is same-step autoreset with no move history: in next-step
    mode or with record_actions it raises instead of leaving pending flags / histories stale,
    and step() after the refused call still matches a fresh env stepped the same way."""
    from acx.envs.ac_env import VecACEnv
    B, L = 256, 36
    acts = torch.randint(0, 12, (4, B), dtype=torch.int32, device=DEV)
    a = VecACEnv(_starts(L, B), horizon_length=3, device=DEV, autoreset_mode="next_step")
    b = VecACEnv(_starts(L, B), horizon_length=3, device=DEV, autoreset_mode="next_step")
    a.step(acts[0])
    b.step(acts[0])
    with pytest.raises(ValueError):
        a.rollout(acts[1:3])
    for t in (1, 2, 3):
        a.step(acts[t])
        b.step(acts[t])
        assert torch.equal(a.state, b.state) and torch.equal(a.pending, b.pending)
    r = VecACEnv(_starts(L, B), device=DEV, record_actions=True)
    with pytest.raises(ValueError):
        r.rollout(acts[:2])


@pytest.mark.parametrize("L", [36, 128])
def test_reset_takes_starting_states_unvalidated(L):
    """reset(options={"starting_states": rows}) copies the rows as the reference's ACEnv.reset
    does (ac_env.py:113-129, no validation); an out-of-domain row is then held as it is and
    reported with err 3 by every step, its exact values kept.  At L = 128 VecACEnv.step
    takes the lengths-carrying kernel (acx_step_lengths, LIVE loads from _row_extent), at L = 36
    acx_step.  An out-of-domain row that only an autoreset brings in (env 20's
    starting row, its episode truncated at the horizon) is taken the same way: the env's row becomes
    that row's exact values, err 3, count 0, and stays so."""
    from acx.envs.ac_env import VecACEnv
    B, H = 128, 3
    env = VecACEnv(_starts(L, B), horizon_length=H, device=DEV)
    rows = _starts(L, B)
    rows[::3] = rows[1]  # no trivial starts: env 20's episode runs to the horizon
    assert rows[5, 2] != 0
    rows[5, 1] = 0  # a zero inside relator 0 (its letters continue after it)
    rows[9, L] = 7  # a letter outside the packed domain
    env.reset(options={"starting_states": rows})
    assert torch.equal(env.state.cpu(), torch.as_tensor(rows))
    bad20 = rows[20].copy()
    bad20[L + 2] = -9  # env 20's starting row, out of the domain; its current row is not
    env.reset_state[20].copy_(torch.as_tensor(bad20))
    g = torch.Generator(device=DEV)
    g.manual_seed(L)
    for t in range(H + 2):
        env.step(torch.randint(0, 12, (B,), dtype=torch.int32, device=DEV, generator=g))
        err = env.err.cpu().numpy()
        st = env.state.cpu().numpy()
        assert err[5] == 3 and err[9] == 3, t
        assert np.array_equal(st[5], rows[5]) and np.array_equal(st[9], rows[9]), t
        if t < H - 1:
            assert err[20] == 0, t
        else:  # step H truncates env 20: autoreset to its out-of-domain starting row
            assert err[20] == 3 and np.array_equal(st[20], bad20), t
            assert int(env.step_count[20].item()) == 0, t
