"""GPU: the rollout's two action paths (int32 ids read in the kernel, acx_rollout; ids
pre-packed 8 per word, acx_pack_actions + acx_rollout_packed) give identical trajectories,
states, step counts and error flags -- including ids outside [0,12), T not a multiple of 8,
partial 64-env tiles and every tile type (L = 36 FastTile, 128 CodeTile, 17 generic) -- and
both equal the oracle env replay."""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


def _starts(L, B, seed=0):
    import acx
    import os
    ms = np.load(os.path.join(os.path.dirname(acx.__file__), "data", "all_presentations.npy"))
    rng = np.random.default_rng(seed)
    out = np.zeros((B, 2 * L), np.int32)
    for i in range(B):
        p = ms[rng.integers(len(ms))]
        a, b = p[:18][p[:18] != 0], p[18:][p[18:] != 0]
        a, b = a[:L], b[:L]
        out[i, : len(a)] = a
        out[i, L : L + len(b)] = b
    return out


def _roll(starts, acts, L, H, cyc, pack, count0=None, resets=None, obs_dtype=torch.int32):
    from acx import ops
    T, B = acts.shape
    st = torch.as_tensor(starts).to(DEV)
    rs = st.clone() if resets is None else torch.as_tensor(resets).to(DEV)
    cnt = (torch.zeros(B, dtype=torch.int32, device=DEV) if count0 is None
           else torch.as_tensor(count0.astype(np.int32)).to(DEV))
    obs = torch.full((T, B, 2 * L), -7, dtype=obs_dtype, device=DEV)
    rew = torch.zeros((T, B), dtype=torch.int32, device=DEV)
    dn = torch.zeros((T, B), dtype=torch.uint8, device=DEV)
    tr = torch.zeros((T, B), dtype=torch.uint8, device=DEV)
    err = torch.zeros(B, dtype=torch.uint8, device=DEV)
    ec = torch.zeros(1, dtype=torch.int32, device=DEV)
    ops.rollout(st, torch.as_tensor(acts).to(DEV), rs, cnt, horizon=H, cyclical=cyc, obs_traj=obs, reward_traj=rew,
                done_traj=dn, trunc_traj=tr, err=err, err_count=ec, pack_actions=pack)
    return [x.cpu().numpy() for x in (st, cnt, obs, rew, dn, tr, err, ec)]


@pytest.mark.parametrize("L,B,T", [(36, 1000, 13), (36, 4096, 40), (128, 200, 21), (17, 333, 9), (36, 64, 1)])
@pytest.mark.parametrize("cyc", [True, False])
def test_packed_equals_unpacked_and_oracle(L, B, T, cyc):
    rng = np.random.default_rng(L * 1000 + T)
    starts = _starts(L, B, seed=T)
    acts = rng.integers(0, 12, size=(T, B)).astype(np.int32)
    a = _roll(starts, acts, L, 5, cyc, pack=False)
    b = _roll(starts, acts, L, 5, cyc, pack=True)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    # oracle replay of the same episode stream (same-step autoreset to the starting state)
    st = starts.copy()
    cnt = np.zeros(B, np.int32)
    for t in range(T):
        r, d, tr, e, _, _ = O.env_step(st, acts[t], L, 5, cnt, reset_state=starts, cyclical=cyc)
        assert np.array_equal(a[2][t], st), t
        assert np.array_equal(a[3][t], r) and np.array_equal(a[4][t], d) and np.array_equal(a[5][t], tr)
    assert int(a[7][0]) == 0


@pytest.mark.parametrize("L", [36, 128])
def test_invalid_ids_same_on_both_paths(L):
    B, T = 300, 19
    rng = np.random.default_rng(5)
    starts = _starts(L, B, seed=1)
    acts = rng.integers(0, 12, size=(T, B)).astype(np.int32)
    bad = rng.random((T, B)) < 0.02
    acts[bad] = rng.choice(np.array([12, 15, 16, -1, 1 << 20, -(1 << 31), 255], np.int32), size=int(bad.sum()))
    a = _roll(starts, acts, L, 7, True, pack=False)
    b = _roll(starts, acts, L, 7, True, pack=True)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    hit = bad.any(0)
    assert (a[6][hit] == 4).all() and (a[6][~hit] == 0).all()
    assert int(a[7][0]) == int(hit.sum())


@pytest.mark.parametrize("B", [777, 1024])  # scalar and 16-byte-vector packing paths
def test_pack_actions_layout(B):
    from acx import _lib
    lib = _lib.load()
    T = 21
    rng = np.random.default_rng(2)
    acts = rng.integers(-3, 20, size=(T, B)).astype(np.int32)
    words = (T + 7) // 8
    assert lib.acx_packed_actions_words(T, B) == words * B
    packed = torch.zeros((words, B), dtype=torch.int32, device=DEV)
    a = torch.as_tensor(acts).to(DEV)
    st = lib.acx_pack_actions(a.data_ptr(), packed.data_ptr(), T, B, torch.cuda.current_stream().cuda_stream)
    assert st == 0
    got = packed.cpu().numpy().view(np.uint32)
    ids = np.where((acts >= 0) & (acts < 12), acts, 15).astype(np.uint32)
    want = np.zeros((words, B), np.uint32)
    for t in range(T):
        want[t // 8] |= ids[t] << np.uint32(4 * (t % 8))
    assert np.array_equal(got, want)


def _trivial_starts(L, B):
    t = np.zeros((8, 2 * L), np.int32)
    for r, (a0, a1) in enumerate([(1, 2), (1, -2), (-1, 2), (-1, -2), (2, 1), (2, -1), (-2, 1), (-2, -1)]):
        t[r, 0], t[r, L] = a0, a1
    return t[np.arange(B) % 8]


@pytest.mark.parametrize("L,B,T,H", [(36, 4096, 40, 5), (36, 4096, 60, 50), (36, 1000, 30, 13), (128, 700, 25, 7),
                                     (17, 333, 20, 9)])
@pytest.mark.parametrize("kind", ["ms", "trivial"])
def test_desynchronised_resets_equal_oracle(L, B, T, H, kind):
    """Episodes out of phase (step_count[i] = i mod H): on every step a scattered subset of each
    wave resets -- a few lanes (each reads its own starting row) or many (the wave reloads its
    tile) -- and, with trivial starts, dones fire on a large share of steps.  Both action paths
    equal the oracle's env replay step by step."""
    rng = np.random.default_rng(L + T + H)
    starts = _starts(L, B, seed=H) if kind == "ms" else _trivial_starts(L, B)
    count0 = (np.arange(B) % H).astype(np.int32)
    acts = rng.integers(0, 12, size=(T, B)).astype(np.int32)
    a = _roll(starts, acts, L, H, True, pack=False, count0=count0)
    b = _roll(starts, acts, L, H, True, pack=True, count0=count0)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    st = starts.copy()
    cnt = count0.copy()
    n_reset = 0
    for t in range(T):
        r, d, tr, e, _, _ = O.env_step(st, acts[t], L, H, cnt, reset_state=starts, cyclical=True)
        n_reset += int((d | tr).sum())
        assert np.array_equal(a[2][t], st), t
        assert np.array_equal(a[3][t], r) and np.array_equal(a[4][t], d) and np.array_equal(a[5][t], tr)
    assert np.array_equal(a[0], st) and np.array_equal(a[1], cnt)
    assert int(a[7][0]) == 0 and n_reset > T


@pytest.mark.parametrize("L", [36, 128, 17])
def test_bad_starting_row_fails_env_at_its_reset(L):
    """A starting row outside the domain is found when the env resets to it: err = 3
    (ACX_ERR_DOMAIN), the env then holds that row (exact values) with step count 0 and never
    moves again; other envs are unaffected (tests/test_gpu_rollout_errors.py has the whole
    contract)."""
    B, T, H = 256, 12, 4
    starts = _starts(L, B, seed=3)
    resets = starts.copy()
    resets[5, 0] = 3          # a letter outside {-2..2}
    resets[70, L + 1] = 0     # a zero inside r1 ...
    resets[70, L + 2] = 1
    count0 = (np.arange(B) % H).astype(np.int32)
    rng = np.random.default_rng(9)
    acts = rng.integers(0, 12, size=(T, B)).astype(np.int32)
    for pack in (False, True):
        st, cnt, obs, rew, dn, tr, err, ec = _roll(starts, acts, L, H, True, pack=pack, count0=count0, resets=resets)
        assert err[5] == 3 and err[70] == 3 and int(ec[0]) == 2
        assert (np.delete(err, [5, 70]) == 0).all()
        assert np.array_equal(st[5], resets[5]) and np.array_equal(st[70], resets[70])
        assert cnt[5] == 0 and cnt[70] == 0
        good = np.setdiff1d(np.arange(B), [5, 70])
        o_st = starts.copy()
        o_cnt = count0.copy()
        for t in range(T):
            O.env_step(o_st, acts[t], L, H, o_cnt, reset_state=resets, cyclical=True)
            assert np.array_equal(obs[t][good], o_st[good]), t
        assert np.array_equal(st[good], o_st[good])


@pytest.mark.parametrize("L,H", [(36, 5), (36, 60), (128, 7), (17, 9)])
def test_step_api_desynchronised_resets_equal_oracle(L, H):
    """acx_step with step_count[i] = i mod H: the per-lane and whole-tile reset paths and
    final_observation, every step against the oracle."""
    from acx import ops
    B, T = 3000, 25
    rng = np.random.default_rng(H)
    starts = _starts(L, B, seed=H)
    count0 = (np.arange(B) % H).astype(np.int32)
    st = torch.as_tensor(starts).to(DEV)
    rs = st.clone()
    cnt = torch.as_tensor(count0).to(DEV)
    rew = torch.zeros(B, dtype=torch.int32, device=DEV)
    dn = torch.zeros(B, dtype=torch.uint8, device=DEV)
    tr = torch.zeros(B, dtype=torch.uint8, device=DEV)
    lens = torch.zeros((B, 2), dtype=torch.int32, device=DEV)
    fo = torch.zeros_like(st)
    err = torch.zeros(B, dtype=torch.uint8, device=DEV)
    o_st = starts.copy()
    o_cnt = count0.copy()
    for t in range(T):
        a = rng.integers(0, 12, size=B).astype(np.int32)
        ops.step(st, torch.as_tensor(a).to(DEV), state_out=st, reset_state=rs, step_count=cnt, horizon=H,
                 cyclical=True, reward=rew, done=dn, truncated=tr, lengths=lens, final_obs=fo, err=err)
        r, d, trn, e, o_len, o_fo = O.env_step(o_st, a, L, H, o_cnt, reset_state=starts, cyclical=True,
                                               want_final=True)
        assert np.array_equal(st.cpu().numpy(), o_st), t
        assert np.array_equal(cnt.cpu().numpy(), o_cnt), t
        assert np.array_equal(rew.cpu().numpy(), r) and np.array_equal(dn.cpu().numpy(), d)
        assert np.array_equal(tr.cpu().numpy(), trn) and np.array_equal(lens.cpu().numpy(), o_len)
        fin = (d | trn).astype(bool)
        assert np.array_equal(fo.cpu().numpy()[fin], o_fo[fin]), t
        assert (err.cpu().numpy() == 0).all()


@pytest.mark.parametrize("L,B,T", [(36, 1000, 13), (36, 333, 11), (36, 4096, 40), (128, 200, 21), (17, 333, 9),
                                   (36, 64, 1)])
@pytest.mark.parametrize("pack", [True, False])
def test_int8_obs_trajectory_equals_int32(L, B, T, pack):
    """acx_rollout_obs8 (the observation trajectory in the reference's int8 observation dtype,
    ac_env.py:64-70): the same episodes as the int32 trajectory, letter for letter, including an
    odd batch at L = 36 (tiles not 16-byte aligned: dword stores), partial tiles, the generic-L
    tile and desynchronised resets."""
    rng = np.random.default_rng(L * 7 + T + B)
    starts = _starts(L, B, seed=B)
    acts = rng.integers(0, 12, size=(T, B)).astype(np.int32)
    count0 = (np.arange(B) % 5).astype(np.int32)
    a = _roll(starts, acts, L, 5, True, pack=pack, count0=count0)
    b = _roll(starts, acts, L, 5, True, pack=pack, count0=count0, obs_dtype=torch.int8)
    assert b[2].dtype == np.int8
    assert np.array_equal(a[2], b[2].astype(np.int32))
    for i in (0, 1, 3, 4, 5, 6, 7):
        assert np.array_equal(a[i], b[i]), i


@pytest.mark.parametrize("pack", [None, True, False])
@pytest.mark.parametrize("L,obs_dtype", [(36, torch.int32), (36, torch.int8), (128, torch.int32)])
def test_rollout_plan_equals_rollout_over_consecutive_launches(L, obs_dtype, pack):
    """ops.RolloutPlan (checks/pointers resolved once, reused buffers) launched three times in a
    row gives the same states, counts, trajectories and errors as ops.rollout per chunk."""
    from acx import ops
    B, T, H = 777, 11, 6
    rng = np.random.default_rng(L)
    starts = torch.as_tensor(_starts(L, B, seed=3)).to(DEV)
    acts = torch.as_tensor(rng.integers(0, 12, size=(3 * T, B)).astype(np.int32)).to(DEV)

    def bufs():
        return dict(obs_traj=torch.full((T, B, 2 * L), -7, dtype=obs_dtype, device=DEV),
                    reward_traj=torch.zeros((T, B), dtype=torch.int32, device=DEV),
                    done_traj=torch.zeros((T, B), dtype=torch.uint8, device=DEV),
                    trunc_traj=torch.zeros((T, B), dtype=torch.uint8, device=DEV),
                    err=torch.zeros(B, dtype=torch.uint8, device=DEV), err_count=torch.zeros(1, dtype=torch.int32,
                                                                                             device=DEV))
    st_a, cnt_a, ba = starts.clone(), torch.zeros(B, dtype=torch.int32, device=DEV), bufs()
    st_b, cnt_b, bb = starts.clone(), torch.zeros(B, dtype=torch.int32, device=DEV), bufs()
    plan = ops.RolloutPlan(st_b, starts, cnt_b, T=T, horizon=H, cyclical=True, pack_actions=pack, **bb)
    assert plan.packs == (ops.packs_actions(T, bb["obs_traj"]) if pack is None else pack)
    for k in range(3):
        a = acts[k * T:(k + 1) * T]
        ops.rollout(st_a, a, starts, cnt_a, horizon=H, cyclical=True, pack_actions=not plan.packs, **ba)
        plan(a)
        torch.cuda.synchronize()
        assert torch.equal(st_a, st_b) and torch.equal(cnt_a, cnt_b), k
        for n in ba:
            assert torch.equal(ba[n], bb[n]), (k, n)
    with pytest.raises(ValueError):
        plan(acts[: T + 1])
    with pytest.raises(ValueError):
        plan(acts[:T].to(torch.int64))
    with pytest.raises(ValueError):
        plan(acts[:T].t().contiguous().t())
