"""GPU parity: the HIP kernels (through libacx.so) against the reference-pinned fixtures and
the CPU oracle, bit-exact.  Needs an MI355X: run with `pytest -m gpu`."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import env_step_contract, GOLDEN
from oracle import oracle as O

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


def _load(name):
    return np.load(os.path.join(GOLDEN, name))


def _gpu_move(states, actions, L, cyc):
    import acx
    s = torch.as_tensor(np.ascontiguousarray(states, dtype=np.int32)).to(DEV)
    a = torch.as_tensor(np.ascontiguousarray(actions, dtype=np.int32)).to(DEV)
    B = s.shape[0]
    lens = torch.empty((B, 2), dtype=torch.int32, device=DEV)
    err = torch.empty((B,), dtype=torch.uint8, device=DEV)
    out = acx.ops.step(s, a, cyclical=bool(cyc), lengths=lens, err=err)
    return out.cpu().numpy(), lens.cpu().numpy(), err.cpu().numpy()


def _has_inner_zero(states, L):
    bad = np.zeros(states.shape[0], bool)
    for h in range(2):
        half = states[:, h * L : (h + 1) * L]
        nz = half != 0
        n = nz.sum(1)
        idx = np.arange(L)[None, :]
        bad |= (nz & (idx >= n[:, None])).any(1)
    return bad


@pytest.mark.parametrize("L", [7, 18, 36, 128])
@pytest.mark.parametrize("cyc", [1, 0])
def test_transitions_fixture(L, cyc):
    d = _load("transitions.npz")
    k = f"L{L}_c{cyc}_"
    out, lens, err = _gpu_move(d[k + "state_in"], d[k + "action"], L, cyc)
    assert np.array_equal(err, d[k + "err"].astype(np.uint8))
    ok = err == 0
    assert np.array_equal(out[ok], d[k + "state_out"][ok].astype(np.int32))
    assert np.array_equal(lens[ok], d[k + "lengths"][ok].astype(np.int32))
    # an env with err keeps its input
    assert np.array_equal(out[~ok], d[k + "state_in"][~ok].astype(np.int32))


@pytest.mark.parametrize("L", [7, 18, 36, 128])
@pytest.mark.parametrize("cyc", [1, 0])
def test_transitions_fixture_in_place(L, cyc):
    """In place (state_out == state_in) the step kernel writes back only the relators that
    changed: every row must still end as the reference's output, failed rows as their input."""
    import acx
    d = _load("transitions.npz")
    k = f"L{L}_c{cyc}_"
    st = torch.as_tensor(d[k + "state_in"].astype(np.int32)).to(DEV)
    a = torch.as_tensor(d[k + "action"].astype(np.int32)).to(DEV)
    err = torch.empty((st.shape[0],), dtype=torch.uint8, device=DEV)
    acx.ops.step(st, a, state_out=st, cyclical=bool(cyc), err=err)
    out, e = st.cpu().numpy(), err.cpu().numpy()
    ok = e == 0
    assert np.array_equal(e, d[k + "err"].astype(np.uint8))
    assert np.array_equal(out[ok], d[k + "state_out"][ok].astype(np.int32))
    assert np.array_equal(out[~ok], d[k + "state_in"][~ok].astype(np.int32))


@pytest.mark.parametrize("L", [36, 128])
def test_in_place_random_walk_with_bad_rows(L):
    """In-place steps over a random walk where some rows are out of the packed domain (letter 3),
    some moves are invalid ids and many envs reset together (horizon 4, synchronised counts:
    whole-tile reloads), every step against the oracle."""
    import acx
    B, T, H = 64 * 9 + 13, 10, 4
    rng = np.random.default_rng(L)
    ms = np.load(os.path.join(os.path.dirname(acx.__file__), "data", "all_presentations.npy"))
    s = np.zeros((B, 2 * L), np.int32)
    for i in range(B):
        p = ms[(7 * i) % len(ms)]
        s[i, :18], s[i, L : L + 18] = p[:18], p[18:]
    bad_rows = rng.choice(B, size=17, replace=False)
    s[bad_rows, 0] = 3
    st = torch.as_tensor(s).to(DEV)
    rs = torch.as_tensor(s).to(DEV)
    cnt = torch.zeros(B, dtype=torch.int32, device=DEV)
    err = torch.zeros(B, dtype=torch.uint8, device=DEV)
    o_st, o_cnt = s.copy(), np.zeros(B, np.int32)
    is_bad = np.zeros(B, bool)
    is_bad[bad_rows] = True
    for t in range(T):
        a = rng.integers(0, 12, size=B).astype(np.int32)
        a[rng.choice(B, size=5, replace=False)] = 12  # invalid move id
        acx.ops.step(st, torch.as_tensor(a).to(DEV), state_out=st, reset_state=rs, step_count=cnt, horizon=H,
                     cyclical=True, err=err)
        # failed envs (out-of-domain row: err 3, bad move id: err 4) keep state and count
        fail = is_bad | (a == 12)
        g = ~fail
        sub, sub_cnt = np.ascontiguousarray(o_st[g]), np.ascontiguousarray(o_cnt[g])
        O.env_step(sub, a[g], L, H, sub_cnt, reset_state=np.ascontiguousarray(s[g]), cyclical=True)
        o_st[g], o_cnt[g] = sub, sub_cnt
        e = err.cpu().numpy()
        assert (e[is_bad] == 3).all() and (e[~is_bad & (a == 12)] == 4).all() and (e[g] == 0).all(), t
        assert np.array_equal(st.cpu().numpy(), o_st), t
        assert np.array_equal(cnt.cpu().numpy(), o_cnt), t


@pytest.mark.parametrize("L", range(1, 10))
def test_smallL_fixture_including_errors(L):
    d = _load("smallL_random.npz")
    s, a, c = d[f"L{L}_state_in"], d[f"L{L}_action"], d[f"L{L}_cyclical"]
    exp_out, exp_len, exp_err = d[f"L{L}_state_out"], d[f"L{L}_lengths"], d[f"L{L}_err"]
    inner = _has_inner_zero(s, L)
    for cyc in (0, 1):
        m = c == cyc
        out, lens, err = _gpu_move(s[m], a[m], L, cyc)
        dom = ~inner[m]
        # inside the domain: identical outputs and identical error classes
        assert np.array_equal(err[dom], exp_err[m][dom].astype(np.uint8))
        ok = dom & (err == 0)
        assert np.array_equal(out[ok], exp_out[m][ok].astype(np.int32))
        assert np.array_equal(lens[ok], exp_len[m][ok].astype(np.int32))
        # zeros inside a relator: flagged, input untouched
        assert (err[~dom] == 3).all()
        assert np.array_equal(out[~dom], s[m][~dom].astype(np.int32))


@pytest.mark.parametrize("L", [2, 5, 13, 16, 17, 36, 47, 64, 65, 100, 128])
@pytest.mark.parametrize("cyc", [1, 0])
def test_random_walks_vs_oracle(L, cyc):
    """Random walks from random (partly unreduced) states, every step checked against the oracle."""
    rng = np.random.default_rng(L * 10 + cyc)
    B = 4096
    s = np.zeros((B, 2 * L), np.int32)
    for b in range(B):
        for h in range(2):
            n = int(rng.integers(1, L + 1))
            s[b, h * L : h * L + n] = rng.choice([1, -1, 2, -2], size=n)
    for t in range(6):
        a = rng.integers(0, 12, size=B).astype(np.int32)
        exp, elen, eerr = O.move_batch(s, a, L, cyc)
        out, lens, err = _gpu_move(s, a, L, cyc)
        assert np.array_equal(err, eerr), t
        assert np.array_equal(out, exp), t
        ok = err == 0
        assert np.array_equal(lens[ok], elen[ok])
        s = exp


def test_bad_action_and_domain_errors():
    L = 4
    s = np.array([[1, 2, 0, 0, -1, 0, 0, 0]] * 4, np.int32)
    out, lens, err = _gpu_move(s, [12, -1, 3, 7], L, 1)
    assert err.tolist()[:2] == [4, 4]
    s2 = np.array([[1, 3, 0, 0, -1, 0, 0, 0], [1, 0, 0, 0, -1, 0, 0, 0],
                   [1, 2, 0, 0, 700, 0, 0, 0], [1, 0, 2, 0, -1, 0, 0, 0]], np.int32)
    out, lens, err = _gpu_move(s2, [0, 0, 0, 0], L, 1)
    # row 1: r1 <- r1 r0 = x^-1 x empties r1 -> reference AssertionError (err 1)
    assert err.tolist() == [3, 1, 3, 3]
    exp, _, eerr = O.move_batch(s2[1:2], [0], L, 1)
    assert eerr[0] == 1
    assert np.array_equal(out[[0, 2, 3]], s2[[0, 2, 3]])


def test_expand12_goldens_and_keys():
    import acx
    d = _load("expand12.npz")
    for tag, L in (("AK3_L36", 36), ("AK2_L7", 7)):
        par = torch.as_tensor(d[tag + "_parents"].astype(np.int32)).to(DEV)
        res = acx.ops.expand12(par, cyclical=False, keys=True)
        assert not res["err"].any()
        assert np.array_equal(res["children"].cpu().numpy(), d[tag + "_children"].astype(np.int32))
        assert np.array_equal(res["lengths"].cpu().numpy(), d[tag + "_lengths"].astype(np.int32))
        back, lens = acx.ops.unpack_keys(res["keys"].reshape(-1, res["keys"].shape[-1]), L, lengths=True)
        assert torch.equal(back, res["children"].reshape(-1, 2 * L))
        assert torch.equal(lens, res["lengths"].reshape(-1, 2))
        # equal keys <=> equal states
        k = res["keys"].reshape(-1, res["keys"].shape[-1]).cpu().numpy()
        c = res["children"].reshape(-1, 2 * L).cpu().numpy()
        _, ik = np.unique(k, axis=0, return_inverse=True)
        _, ic = np.unique(c, axis=0, return_inverse=True)
        ik, ic = ik.reshape(-1), ic.reshape(-1)
        pairs = np.unique(np.stack([ik, ic], 1), axis=0)
        assert len(pairs) == len(np.unique(ik)) == len(np.unique(ic))


@pytest.mark.parametrize("L", [7, 36, 128])
@pytest.mark.parametrize("cyc", [0, 1])
def test_expand12_vs_oracle(L, cyc):
    import acx
    rng = np.random.default_rng(L + cyc)
    N = 1000
    s = np.zeros((N, 2 * L), np.int32)
    for b in range(N):
        for h in range(2):
            n = int(rng.integers(1, L + 1))
            s[b, h * L : h * L + n] = rng.choice([1, -1, 2, -2], size=n)
    ch, lens, err = O.expand12(s, L, cyc)
    res = acx.ops.expand12(torch.as_tensor(s).to(DEV), cyclical=bool(cyc), keys=True)
    assert np.array_equal(res["err"].cpu().numpy(), err)
    assert np.array_equal(res["children"].cpu().numpy(), ch)
    ok = err == 0
    assert np.array_equal(res["lengths"].cpu().numpy()[ok], lens[ok])


@pytest.mark.parametrize("L,N", [(36, 64 * 5 + 17), (128, 64 * 3 + 1), (17, 333), (36, 64)])
def test_expand12_children_with_bad_parents(L, N):
    """Block-per-tile children kernel: children, lengths and error codes of every (parent,
    action) against the oracle, partial tiles, children without keys, and out-of-domain parents
    (a letter 3, or a zero inside a relator -- which CodeTile's code slots cannot hold: every
    child is err 3 and an exact copy of the parent row)."""
    import acx
    rng = np.random.default_rng(L * 31 + N)
    s = np.zeros((N, 2 * L), np.int32)
    for b in range(N):
        for h in range(2):
            n = int(rng.integers(3, L + 1))
            s[b, h * L : h * L + n] = rng.choice([1, -1, 2, -2], size=n)
    bad = rng.choice(N, size=max(2, N // 40), replace=False)
    s[bad[::2], 0] = 3
    s[bad[1::2], 1] = 0  # a zero inside r0
    good = np.ones(N, bool)
    good[bad] = False
    ch, lens, err = O.expand12(np.ascontiguousarray(s[good]), L, False)
    res = acx.ops.expand12(torch.as_tensor(s).to(DEV), cyclical=False)
    g_ch, g_len, g_err = (res[k].cpu().numpy() for k in ("children", "lengths", "err"))
    assert np.array_equal(g_err[good], err)
    assert np.array_equal(g_ch[good], ch)
    ok = err == 0
    assert np.array_equal(g_len[good][ok], lens[ok])
    assert (g_err[bad] == 3).all()
    assert np.array_equal(g_ch[bad], np.repeat(s[bad][:, None, :], 12, axis=1))


@pytest.mark.parametrize("L", [36, 128, 17])
def test_canonicalize_out_of_domain_rows_exact(L):
    """acx_canonicalize leaves rows outside the packed domain exactly as they are (err 3): a letter
    3 and a zero inside a relator (the latter is not flagged by the tile load, and CodeTile's code
    slots cannot hold it) -- in place and out of place."""
    import acx
    rng = np.random.default_rng(L + 5)
    B = 64 * 3 + 7
    s = np.zeros((B, 2 * L), np.int32)
    for b in range(B):
        for h in range(2):
            n = int(rng.integers(3, L + 1))
            s[b, h * L : h * L + n] = rng.choice([1, -1, 2, -2], size=n)
    bad = rng.choice(B, size=12, replace=False)
    s[bad[:6], L] = 3
    s[bad[6:], L + 1] = 0
    t = torch.as_tensor(s).to(DEV)
    out, lens, err = acx.ops.canonicalize(t, cyclical=True)
    o, e = out.cpu().numpy(), err.cpu().numpy()
    assert (e[bad] == 3).all() and np.array_equal(o[bad], s[bad])
    out2, _, err2 = acx.ops.canonicalize(t, cyclical=True, out=t)
    assert np.array_equal(t.cpu().numpy()[bad], s[bad]) and torch.equal(err2, err)


@pytest.mark.parametrize("L", [3, 36, 128])
def test_canonicalize_vs_oracle(L):
    import acx
    rng = np.random.default_rng(L)
    B = 2000
    s = np.zeros((B, 2 * L), np.int32)
    for b in range(B):
        for h in range(2):
            n = int(rng.integers(0 if b % 50 == 0 else 1, L + 1))
            s[b, h * L : h * L + n] = rng.choice([1, -1, 2, -2], size=n)
    for cyc in (0, 1):
        out, lens, err = acx.ops.canonicalize(torch.as_tensor(s).to(DEV), cyclical=bool(cyc))
        out, lens, err = out.cpu().numpy(), lens.cpu().numpy(), err.cpu().numpy()
        for b in range(B):
            e, le, ee = O.simplify_presentation(s[b], L, cyc)
            assert err[b] == ee, b
            if ee == 0:
                assert np.array_equal(out[b], e) and lens[b].tolist() == le


def test_kat_paths_through_acmove():
    from acx import ACMove
    from acx.envs.utils import is_presentation_trivial
    with open(os.path.join(GOLDEN, "kat_paths.json")) as f:
        paths = json.load(f)
    for p in paths:
        # long paths replayed in one batched walk: a (1, 2L) state stepped len(actions) times
        L = p["L"]
        s = np.array(p["start"], np.int64)
        totals = []
        if len(p["actions"]) <= 60:
            for a in p["actions"]:
                s, lens = ACMove(a, s, L, None, cyclical=bool(p["cyclical"]))
                totals.append(sum(lens))
        else:
            st = s.astype(np.int32)[None]
            for a in p["actions"]:
                st, lens, err = _gpu_move(st, [a], L, p["cyclical"])
                assert err[0] == 0
                totals.append(int(lens[0].sum()))
            s = st[0]
        assert totals == p["totals"], p["name"]
        assert list(map(int, s)) == p["final"]
        assert is_presentation_trivial(s) == p["trivial"]


def test_env_config1():
    from acx import ACEnv, ACEnvConfig
    with open(os.path.join(GOLDEN, "config1.json")) as f:
        rows = json.load(f)
    for row in rows:
        env = ACEnv(ACEnvConfig(initial_state=[1, 0, 2, 0]))
        env.reset()
        s, r, d, tr, info = env.step(row["action"])
        assert s.tolist() == row["state"]
        assert (r, d, tr) == (row["reward"], row["done"], row["truncated"])
        assert {k: list(v) for k, v in info.items()} == row["info"]
        assert env.lengths == row["lengths"]


def test_vec_env_episodes_fixture():
    """VecACEnv.step (same-step autoreset) against ACEnv episodes run by the reference."""
    from acx import VecACEnv
    d = _load("env_episodes.npz")
    env = VecACEnv(d["initial"].astype(np.int32), horizon_length=int(d["horizon"]), device=DEV)
    for t in range(d["actions"].shape[0]):
        obs, rew, done, trunc, info = env.step(torch.as_tensor(d["actions"][t].astype(np.int32)).to(DEV))
        assert np.array_equal(rew.cpu().numpy(), d["reward"][t]), t
        assert np.array_equal(done.cpu().numpy(), d["done"][t].astype(np.uint8)), t
        assert np.array_equal(trunc.cpu().numpy(), d["truncated"][t].astype(np.uint8)), t
        assert np.array_equal(obs.cpu().numpy(), d["obs"][t].astype(np.int32)), t
        m = (d["done"][t] | d["truncated"][t]).astype(bool)
        assert np.array_equal(info["final_observation"].cpu().numpy()[m], d["final_obs"][t][m].astype(np.int32))
    assert int(env.err_count.item()) == 0


@pytest.mark.parametrize("fmt", ["final_info", "actions"])
def test_vec_env_info_actions_contract(fmt):
    """record_actions: the info dict training.py:273-280 reads for solved episodes.  Expected move
    lists follow ACEnv's own bookkeeping over the reference's episodes (env_episodes.npz):
    `self.actions += [action]` per step, cleared by reset (ac_env.py:92,105-110,124)."""
    from acx import VecACEnv
    d = _load("env_episodes.npz")
    T, B = d["actions"].shape
    env = VecACEnv(d["initial"].astype(np.int32), horizon_length=int(d["horizon"]), device=DEV,
                   record_actions=True, info_format=fmt)
    hist = [[] for _ in range(B)]
    n_solved = 0
    for t in range(T):
        obs, rew, done, trunc, info = env.step(torch.as_tensor(d["actions"][t].astype(np.int32)).to(DEV))
        assert np.array_equal(obs.cpu().numpy(), d["obs"][t].astype(np.int32)), t
        dn, tr = d["done"][t].astype(bool), d["truncated"][t].astype(bool)
        for i in range(B):
            hist[i].append(int(d["actions"][t][i]))
        if not (dn | tr).any():
            assert info.keys() <= {"final_observation"}, t
        for i in range(B):
            if fmt == "final_info":
                if dn[i] or tr[i]:
                    assert info["_final_info"][i] and info["_final_observation"][i]
                    # training.py:276-277
                    assert info["final_info"][i] == ({"actions": hist[i]} if dn[i] else {}), (t, i)
                elif "final_info" in info:
                    assert not info["_final_info"][i] and info["final_info"][i] is None
            elif dn[i]:
                assert info["_actions"][i] and list(info["actions"][i]) == hist[i], (t, i)  # training.py:280
            elif "actions" in info:
                assert not info["_actions"][i]
            if dn[i] or tr[i]:
                n_solved += int(dn[i])
                hist[i] = []
    assert n_solved > 0


def test_rollout_equals_repeated_step_and_fixture():
    from acx import VecACEnv
    d = _load("env_episodes.npz")
    L, H = int(d["L"]), int(d["horizon"])
    init = d["initial"].astype(np.int32)
    acts = torch.as_tensor(d["actions"].astype(np.int32)).to(DEV)
    T, B = acts.shape
    env = VecACEnv(init, horizon_length=H, device=DEV)
    obs = torch.empty((T, B, 2 * L), dtype=torch.int32, device=DEV)
    rew = torch.empty((T, B), dtype=torch.int32, device=DEV)
    dn = torch.empty((T, B), dtype=torch.uint8, device=DEV)
    tr = torch.empty((T, B), dtype=torch.uint8, device=DEV)
    # two launches (T/2 each) to also check the carried step_count / state
    env.rollout(acts[: T // 2], obs[: T // 2], rew[: T // 2], dn[: T // 2], tr[: T // 2])
    env.rollout(acts[T // 2 :], obs[T // 2 :], rew[T // 2 :], dn[T // 2 :], tr[T // 2 :])
    assert np.array_equal(obs.cpu().numpy(), d["obs"].astype(np.int32))
    assert np.array_equal(rew.cpu().numpy(), d["reward"])
    assert np.array_equal(dn.cpu().numpy(), d["done"].astype(np.uint8))
    assert np.array_equal(tr.cpu().numpy(), d["truncated"].astype(np.uint8))
    assert int(env.err_count.item()) == 0


def _ms_starts(L, B):
    import acx
    ms = np.load(os.path.join(os.path.dirname(acx.__file__), "data", "all_presentations.npy"))
    out = np.zeros((B, 2 * L), np.int32)
    for i in range(B):
        p = ms[i % len(ms)]
        a, b = p[:18][p[:18] != 0], p[18:][p[18:] != 0]
        out[i, : len(a)] = a
        out[i, L : L + len(b)] = b
    return out


@pytest.mark.parametrize("L", [36, 128])
def test_full_size_rollout_properties_and_sampled_parity(L):
    """Full per-GPU batch (2^20 envs: config 3 at L=36, config 5's shard at L=128):
    size-independent invariants on every env (valid, freely + cyclically reduced, lengths =
    letter counts) and bit-exact oracle replay of a sample of envs."""
    from acx import VecACEnv
    B = 1 << 20
    T, H = 24, 10
    init = _ms_starts(L, B)
    env = VecACEnv(init, horizon_length=H, device=DEV, track_final_obs=False)
    g = torch.Generator(device=DEV)
    g.manual_seed(0)
    acts = torch.randint(0, 12, (T, B), dtype=torch.int32, device=DEV, generator=g)
    obs = torch.empty((T, B, 2 * L), dtype=torch.int32, device=DEV)
    rew = torch.empty((T, B), dtype=torch.int32, device=DEV)
    dn = torch.empty((T, B), dtype=torch.uint8, device=DEV)
    tr = torch.empty((T, B), dtype=torch.uint8, device=DEV)
    env.rollout(acts, obs, rew, dn, tr)
    assert int(env.err_count.item()) == 0
    # invariants on the final states of every env
    st = env.state
    nz = st != 0
    r0, r1 = st[:, :L], st[:, L:]
    n0, n1 = nz[:, :L].sum(1), nz[:, L:].sum(1)
    idx = torch.arange(L, device=DEV)[None]
    assert not (nz[:, :L] & (idx >= n0[:, None])).any() and not (nz[:, L:] & (idx >= n1[:, None])).any()
    assert (n0 > 0).all() and (n1 > 0).all()
    for r, n in ((r0, n0), (r1, n1)):
        adj = (r[:, :-1] == -r[:, 1:]) & (r[:, :-1] != 0)
        assert not adj.any()
        last = torch.gather(r, 1, (n - 1).clamp(min=0)[:, None])[:, 0]
        assert not ((r[:, 0] == -last) & (n > 1)).any()
    # sampled bit-exact replay
    rng = np.random.default_rng(1)
    sample = rng.choice(B, size=512, replace=False)
    s = init[sample].copy()
    cnt = np.zeros(len(sample), np.int32)
    A = acts[:, torch.as_tensor(sample, device=DEV)].cpu().numpy()
    O_obs = obs[:, torch.as_tensor(sample, device=DEV)].cpu().numpy()
    O_rew = rew[:, torch.as_tensor(sample, device=DEV)].cpu().numpy()
    for t in range(T):
        r, d_, t_, e, _, _ = O.env_step(s, A[t], L, H, cnt, reset_state=init[sample])
        assert not e.any()
        assert np.array_equal(s, O_obs[t]), t
        assert np.array_equal(r, O_rew[t]), t


@pytest.mark.parametrize("L,B", [(36, 1 << 20), (128, 1 << 20), (36, 65536)])
def test_full_size_step_api_in_place(L, B):
    """The per-call step API at full size: 2^20 envs at L = 36 (config 3's
    batch) and L = 128 (config 5's per-GPU shard), and config 2's exact batch (65,536 envs, L =
    36).  24 in-place acx_step calls with autoreset (horizon 10) -- the dirty-relator write-back
    (unchanged relators skipped, partial 64-B lines) -- against, on every env and every step:
    the same steps out of place (every row written), the lengths-carrying in-place steps
    (acx_step_lengths: only live chunks read and written), the fused rollout's observations, rewards,
    done and truncated flags; size-independent invariants (valid, reduced, lengths = letter
    counts); and a 512-env sampled oracle replay of states, counts, rewards and lengths."""
    from acx import ops
    T, H = 24, 10
    init = _ms_starts(L, B)
    starts = torch.as_tensor(init).to(DEV)
    g = torch.Generator(device=DEV)
    g.manual_seed(3)
    acts = torch.randint(0, 12, (T, B), dtype=torch.int32, device=DEV, generator=g)
    # fused rollout of the same stream (its trajectory is the reference for every step)
    st_r, cnt_r = starts.clone(), torch.zeros(B, dtype=torch.int32, device=DEV)
    obs = torch.empty((T, B, 2 * L), dtype=torch.int32, device=DEV)
    rew_r = torch.empty((T, B), dtype=torch.int32, device=DEV)
    dn_r = torch.empty((T, B), dtype=torch.uint8, device=DEV)
    tr_r = torch.empty((T, B), dtype=torch.uint8, device=DEV)
    ops.rollout(st_r, acts, starts, cnt_r, horizon=H, cyclical=True, obs_traj=obs, reward_traj=rew_r, done_traj=dn_r,
                trunc_traj=tr_r)
    st, cnt = starts.clone(), torch.zeros(B, dtype=torch.int32, device=DEV)  # in place
    st_o, cnt_o = starts.clone(), torch.zeros(B, dtype=torch.int32, device=DEV)  # out of place
    st_l, cnt_l = starts.clone(), torch.zeros(B, dtype=torch.int32, device=DEV)  # lengths-carrying
    outs = [{k: torch.empty(B, dtype=dt, device=DEV) for k, dt in
             (("rew", torch.int32), ("dn", torch.uint8), ("tr", torch.uint8), ("err", torch.uint8))} for _ in range(3)]
    for o in outs:
        o["len"] = torch.empty((B, 2), dtype=torch.int32, device=DEV)
        o["ec"] = torch.zeros(1, dtype=torch.int32, device=DEV)
    nz0 = starts.view(B, 2, L) != 0
    outs[2]["len"].copy_(nz0.sum(2).to(torch.int32))  # acx_step_lengths: the rows' lengths carried
    rng = np.random.default_rng(L + B)
    sample = rng.choice(B, size=512, replace=False)
    si = torch.as_tensor(sample, device=DEV)
    s = init[sample].copy()
    o_cnt = np.zeros(len(sample), np.int32)
    idx = torch.arange(L, device=DEV)[None]
    for t in range(T):
        a = acts[t]
        o = outs[0]
        ops.step(st, a, state_out=st, reset_state=starts, step_count=cnt, horizon=H, cyclical=True, reward=o["rew"],
                 done=o["dn"], truncated=o["tr"], lengths=o["len"], err=o["err"], err_count=o["ec"])
        p = outs[1]
        nxt = torch.empty_like(st_o)
        ops.step(st_o, a, state_out=nxt, reset_state=starts, step_count=cnt_o, horizon=H, cyclical=True,
                 reward=p["rew"], done=p["dn"], truncated=p["tr"], lengths=p["len"], err=p["err"], err_count=p["ec"])
        st_o = nxt
        q = outs[2]
        ops.step(st_l, a, state_out=st_l, reset_state=starts, step_count=cnt_l, horizon=H, cyclical=True,
                 reward=q["rew"], done=q["dn"], truncated=q["tr"], lengths=q["len"], err=q["err"], err_count=q["ec"],
                 lengths_in=True)
        assert torch.equal(st, st_o) and torch.equal(cnt, cnt_o), t
        assert torch.equal(st, st_l) and torch.equal(cnt, cnt_l), t
        for k in ("rew", "dn", "tr", "err", "len"):
            assert torch.equal(o[k], p[k]), (t, k)
            assert torch.equal(o[k], q[k]), (t, k)
        assert torch.equal(st, obs[t]), t
        assert torch.equal(o["rew"], rew_r[t]) and torch.equal(o["dn"], dn_r[t]) and torch.equal(o["tr"], tr_r[t]), t
        # invariants on every env
        nz = st != 0
        n0, n1 = nz[:, :L].sum(1), nz[:, L:].sum(1)
        assert not (nz[:, :L] & (idx >= n0[:, None])).any() and not (nz[:, L:] & (idx >= n1[:, None])).any()
        assert (n0 > 0).all() and (n1 > 0).all()
        assert torch.equal(o["len"], torch.stack([n0, n1], 1).to(torch.int32)), t
        for r, n in ((st[:, :L], n0), (st[:, L:], n1)):
            assert not ((r[:, :-1] == -r[:, 1:]) & (r[:, :-1] != 0)).any()
            last = torch.gather(r, 1, (n - 1).clamp(min=0)[:, None])[:, 0]
            assert not ((r[:, 0] == -last) & (n > 1)).any()
        # sampled oracle replay
        r_, d_, tr_, e_, ln_, _ = O.env_step(s, a[si].cpu().numpy(), L, H, o_cnt, reset_state=init[sample])
        assert not e_.any()
        assert np.array_equal(st[si].cpu().numpy(), s) and np.array_equal(cnt[si].cpu().numpy(), o_cnt), t
        assert np.array_equal(o["rew"][si].cpu().numpy(), r_) and np.array_equal(o["len"][si].cpu().numpy(), ln_), t
    assert int(outs[0]["ec"].item()) == 0 and int(outs[1]["ec"].item()) == 0
    assert torch.equal(st, st_r) and torch.equal(cnt, cnt_r)


def test_search_kat_ak2():
    from acx import bfs, greedy_search
    with open(os.path.join(GOLDEN, "kat_search.json")) as f:
        kat = json.load(f)
    ak2 = np.array([1, 1, -2, -2, -2, 0, 0, 1, 2, 1, -2, -1, -2, 0])
    ok, path = bfs(presentation=ak2, max_nodes_to_explore=int(1e6))
    assert [ok, [list(x) for x in path]] == kat["bfs_ak2"]
    assert list(bfs(presentation=ak2, max_nodes_to_explore=10)) == [False, None]
    ok, path = greedy_search(presentation=ak2, max_nodes_to_explore=int(1e6))
    assert [ok, [list(x) for x in path]] == kat["greedy_ak2"]
    ok, path = greedy_search(presentation=ak2, max_nodes_to_explore=10)
    assert [ok, [list(x) for x in path]] == kat["greedy_ak2_budget10"]


def test_search_kat_miller_schupp():
    from acx import bfs, greedy_search
    with open(os.path.join(GOLDEN, "kat_search.json")) as f:
        kat = json.load(f)
    for case in kat["miller_schupp"]:
        fn = greedy_search if case["search_fn"] == "greedy_search" else bfs
        solved, unsolved, paths = [], [], []
        for pres in case["presentations"]:
            ok, path = fn(presentation=np.array(pres), max_nodes_to_explore=case["budget"])
            if ok:
                solved.append(pres)
                paths.append([list(x) for x in path])
            else:
                unsolved.append(pres)
        assert solved == case["solved"], case["search_fn"]
        assert unsolved == case["unsolved"], case["search_fn"]
        assert paths == case["paths"], case["search_fn"]


@pytest.mark.parametrize("L", [36, 128])
@pytest.mark.parametrize("B", [1, 63, 65, 1000, 64 * 7 + 5])
def test_partial_tiles_fast_path(L, B):
    """FastTile (L % 4 == 0) with batches that end in a partial 64-env tile: step, rollout,
    expand12 and canonicalize against the oracle; out-of-place and in-place."""
    import acx
    rng = np.random.default_rng(B * 7 + L)
    s = np.zeros((B, 2 * L), np.int32)
    for b in range(B):
        for h in range(2):
            n = int(rng.integers(1, L + 1))
            s[b, h * L : h * L + n] = rng.choice([1, -1, 2, -2], size=n)
    a = rng.integers(0, 12, size=B).astype(np.int32)
    exp, elen, eerr = O.move_batch(s, a, L, 1)
    out, lens, err = _gpu_move(s, a, L, 1)
    assert np.array_equal(out, exp) and np.array_equal(err, eerr)
    # in place
    st = torch.as_tensor(s).to(DEV)
    acx.ops.step(st, torch.as_tensor(a).to(DEV), state_out=st, cyclical=True)
    assert np.array_equal(st.cpu().numpy(), exp)
    # rollout over 12 steps with autoreset (horizon 5) vs the oracle env
    T, H = 12, 5
    A = rng.integers(0, 12, size=(T, B)).astype(np.int32)
    # starting states must be valid presentations (ACEnvConfig's rule): replace rows whose
    # unreduced input reduced to an empty relator
    empty = (exp[:, :L] != 0).sum(1) == 0
    empty |= (exp[:, L:] != 0).sum(1) == 0
    exp[empty] = 0
    exp[empty, 0] = 1
    exp[empty, L] = 2
    env = acx.VecACEnv(exp, horizon_length=H, device=DEV)
    obs = torch.empty((T, B, 2 * L), dtype=torch.int32, device=DEV)
    rew = torch.empty((T, B), dtype=torch.int32, device=DEV)
    env.rollout(torch.as_tensor(A).to(DEV), obs, rew)
    ost = exp.copy()
    cnt = np.zeros(B, np.int32)
    for t in range(T):  # random states: some moves empty a relator -> the error contract
        r, d, tr, e = env_step_contract(ost, A[t], cnt, exp, L, H)
        assert np.array_equal(obs[t].cpu().numpy(), ost), t
        assert np.array_equal(rew[t].cpu().numpy(), r), t
    assert np.array_equal(env.state.cpu().numpy(), ost)
    assert np.array_equal(env.step_count.cpu().numpy(), cnt)
    # expand12 (keys + children) and canonicalize
    res = acx.ops.expand12(torch.as_tensor(s).to(DEV), cyclical=False, keys=True)
    ch, cl, ce = O.expand12(s, L, False)
    assert np.array_equal(res["children"].cpu().numpy(), ch)
    back = acx.ops.unpack_keys(res["keys"].reshape(-1, res["keys"].shape[-1]), L)
    ok = ce.reshape(-1) == 0
    assert np.array_equal(back.cpu().numpy()[ok], ch.reshape(-1, 2 * L)[ok])
    # an errored child's key is the sentinel: both length bytes 0xFF (acx.h)
    _, blen = acx.ops.unpack_keys(res["keys"].reshape(-1, res["keys"].shape[-1]), L, lengths=True)
    assert (blen.cpu().numpy()[~ok] == 0xFF).all()
    keys_only = acx.ops.expand12(torch.as_tensor(s).to(DEV), cyclical=False, children=False, keys=True)
    assert torch.equal(keys_only["keys"], res["keys"])


def test_api_edge_cases():
    import acx
    from acx import _lib
    L = 36
    s = torch.zeros((0, 2 * L), dtype=torch.int32, device=DEV)
    out = acx.ops.step(s, torch.zeros(0, dtype=torch.int32, device=DEV))
    assert out.shape == (0, 2 * L)
    lib = _lib.load()
    base = torch.zeros((8, 2 * L + 1), dtype=torch.int32, device=DEV)
    bad_ptr = base.data_ptr() + 4  # misaligned
    rc = lib.acx_step(bad_ptr, bad_ptr, base.data_ptr(), None, None, None, None, None, None, None, None, None,
                      4, L, 0, 1, torch.cuda.current_stream().cuda_stream)
    assert rc == _lib.E_ARG
    rc = lib.acx_step(base.data_ptr(), base.data_ptr(), base.data_ptr(), None, None, None, None, None, None, None,
                      None, None, 4, 129, 0, 1, torch.cuda.current_stream().cuda_stream)
    assert rc == _lib.E_ARG
    with pytest.raises(ValueError):
        acx.ops.step(torch.zeros((4, 7), dtype=torch.int32, device=DEV), torch.zeros(4, dtype=torch.int32, device=DEV))
    with pytest.raises(TypeError):
        acx.ops.step(torch.zeros((4, 8), dtype=torch.int64, device=DEV), torch.zeros(4, dtype=torch.int32, device=DEV))


def test_acenv_api_mirrors_reference():
    """ACEnv: reset(options), step returns, truncation at the horizon, info actions, errors."""
    from acx import ACEnv, ACEnvConfig
    env = ACEnv(ACEnvConfig(initial_state=[1, 2, 0, -1, 0, 0], horizon_length=3))
    s, info = env.reset()
    assert s.tolist() == [1, 2, 0, -1, 0, 0] and info == {}
    outs = [env.step(a) for a in (8, 8, 8)]
    assert [o[3] for o in outs] == [False, False, True]
    from oracle import oracle as O
    st = np.array([[1, 2, 0, -1, 0, 0]], np.int32)
    cnt = np.zeros(1, np.int32)
    for a, o in zip((8, 8, 8), outs):
        r, d, tr, e, lens, _ = O.env_step(st, [a], 3, 3, cnt)
        assert o[0].tolist() == st[0].tolist() and o[1] == int(r[0]) and o[2] == bool(d[0])
    s, _ = env.reset(options={"starting_state": np.array([1, 0, 0, 2, 0, 0])})
    assert env.lengths == [1, 1] and env.count_steps == 0
    with pytest.raises(NotImplementedError):
        ACEnv(ACEnvConfig(use_supermoves=True))
    # conjugating an empty relator -> IndexError, emptying a relator -> AssertionError
    from acx import ACMove
    with pytest.raises(IndexError):
        ACMove(7, np.array([0, 0, 1, 0]), 2, None)
    with pytest.raises(AssertionError):
        ACMove(0, np.array([1, 0, -1, 0]), 2, None)


def test_step_api_under_hipgraph_capture():
    """acx_step launches captured into a hipGraph (torch.cuda.CUDAGraph) replay to the same
    states as eager launches: the C-ABI never allocates or synchronises."""
    import acx
    L, B, K = 36, 3000, 12
    rng = np.random.default_rng(5)
    ms = np.load(os.path.join(os.path.dirname(acx.__file__), "data", "all_presentations.npy"))
    init = np.zeros((B, 2 * L), np.int32)
    for i in range(B):
        p = ms[i % len(ms)]
        init[i, :18], init[i, L : L + 18] = p[:18], p[18:]
    acts = torch.as_tensor(rng.integers(0, 12, size=(K, B)).astype(np.int32)).to(DEV)
    rs = torch.as_tensor(init).to(DEV)

    def run(st, cnt, rew):
        for t in range(K):
            acx.ops.step(st, acts[t], state_out=st, reset_state=rs, step_count=cnt, horizon=5, reward=rew[t])

    st_e, cnt_e = rs.clone(), torch.zeros(B, dtype=torch.int32, device=DEV)
    rew_e = torch.zeros((K, B), dtype=torch.int32, device=DEV)
    run(st_e, cnt_e, rew_e)
    st_g, cnt_g = rs.clone(), torch.zeros(B, dtype=torch.int32, device=DEV)
    rew_g = torch.zeros((K, B), dtype=torch.int32, device=DEV)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            run(st_g, cnt_g, rew_g)
    # capture does not execute: reset and replay
    st_g.copy_(rs)
    cnt_g.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(st_g, st_e) and torch.equal(cnt_g, cnt_e) and torch.equal(rew_g, rew_e)


def test_acenv_error_does_not_count_a_step():
    """A move that raises (ac_env.py:93-95 -> utils.py:264-266) happens before count_steps += 1
    (ac_env.py:102): a caller that catches it and keeps stepping truncates at the same step as
    the reference (the device step counter is not advanced either)."""
    import acx
    env = acx.ACEnv(acx.ACEnvConfig(initial_state=np.array([1, 0, 1, 0]), horizon_length=2))
    with pytest.raises(AssertionError):
        env.step(1)  # r0 <- r0 r1^-1 = x x^-1: empty relator
    assert env.count_steps == 0 and env.actions == [1]
    s, r, d, t, info = env.step(4)
    assert not t and env.count_steps == 1
    s, r, d, t, info = env.step(4)
    assert t and env.count_steps == 2


def test_headline_rollout_every_env_vs_oracle():
    """The driver's headline workload exactly (BASELINE configs[2]: bench.py's 2^20 Miller-Schupp
    starts, L = 36, horizon 200, one ops.RolloutPlan launch of K = 20 steps with the full int32
    obs trajectory), checked on EVERY env and step against the C oracle's batched ACEnv.step
    with same-step autoreset: obs rows, rewards, done and truncated flags, final state and counts."""
    import bench
    from acx import ops
    L, B, K, H = 36, 1 << 20, 20, 200
    init = bench.ms_starts(L, B)
    starts = torch.as_tensor(init).to(DEV)
    state = starts.clone()
    cnt = torch.zeros(B, dtype=torch.int32, device=DEV)
    g = torch.Generator(device=DEV)
    g.manual_seed(0)
    acts = torch.randint(0, 12, (K, B), dtype=torch.int32, device=DEV, generator=g)
    obs = torch.empty((K, B, 2 * L), dtype=torch.int32, device=DEV)
    rew = torch.empty((K, B), dtype=torch.int32, device=DEV)
    dn = torch.empty((K, B), dtype=torch.uint8, device=DEV)
    tr = torch.empty((K, B), dtype=torch.uint8, device=DEV)
    err = torch.zeros(B, dtype=torch.uint8, device=DEV)
    ec = torch.zeros(1, dtype=torch.int32, device=DEV)
    plan = ops.RolloutPlan(state, starts, cnt, T=K, horizon=H, cyclical=True, obs_traj=obs, reward_traj=rew,
                           done_traj=dn, trunc_traj=tr, err=err, err_count=ec)
    plan(acts)
    torch.cuda.synchronize()
    s = init.copy()
    c = np.zeros(B, np.int32)
    A = acts.cpu().numpy()
    for t in range(K):
        r, d_, t_, e, _, _ = O.env_step(s, A[t], L, H, c, reset_state=init)
        assert not e.any()
        assert np.array_equal(obs[t].cpu().numpy(), s), t
        assert np.array_equal(rew[t].cpu().numpy(), r), t
        assert np.array_equal(dn[t].cpu().numpy(), d_) and np.array_equal(tr[t].cpu().numpy(), t_), t
    assert np.array_equal(state.cpu().numpy(), s) and np.array_equal(cnt.cpu().numpy(), c)
    assert int(ec.item()) == 0


def test_packed_rollout_full_horizon_every_env_vs_oracle():
    """The packed-move-id rollout path at full size: BASELINE configs[2]'s own
    horizon -- 2^20 Miller-Schupp starts, L = 36, ONE ops.RolloutPlan launch of K = 200 steps with
    the int32 obs trajectory, so the move ids go through acx_pack_actions (ops.packs_actions: an
    int32 trajectory longer than 32 steps).  Against the C oracle's batched ACEnv.step with
    same-step autoreset (training.py:221-356's collection loop): every env's reward / done /
    truncated at every step, the final state and step count of every env (step 200 truncates and
    resets every env whose episode never ended), and the obs rows of a 4,096-env sample at every step."""
    import bench
    from acx import ops
    L, B, K, H = 36, 1 << 20, 200, 200
    assert ops.packs_actions(K, torch.zeros(1, dtype=torch.int32))
    init = bench.ms_starts(L, B)
    starts = torch.as_tensor(init).to(DEV)
    state = starts.clone()
    cnt = torch.zeros(B, dtype=torch.int32, device=DEV)
    g = torch.Generator(device=DEV)
    g.manual_seed(6)
    acts = torch.randint(0, 12, (K, B), dtype=torch.int32, device=DEV, generator=g)
    obs = torch.empty((K, B, 2 * L), dtype=torch.int32, device=DEV)  # 60 GB of HBM
    rew = torch.empty((K, B), dtype=torch.int32, device=DEV)
    dn = torch.empty((K, B), dtype=torch.uint8, device=DEV)
    tr = torch.empty((K, B), dtype=torch.uint8, device=DEV)
    err = torch.zeros(B, dtype=torch.uint8, device=DEV)
    ec = torch.zeros(1, dtype=torch.int32, device=DEV)
    plan = ops.RolloutPlan(state, starts, cnt, T=K, horizon=H, cyclical=True, obs_traj=obs, reward_traj=rew,
                           done_traj=dn, trunc_traj=tr, err=err, err_count=ec)
    plan(acts)
    torch.cuda.synchronize()
    sample = torch.as_tensor(np.random.default_rng(6).choice(B, 4096, replace=False)).to(DEV)
    obs_s = obs[:, sample].cpu().numpy()
    del obs
    sample = sample.cpu().numpy()
    R, D, T, A = rew.cpu().numpy(), dn.cpu().numpy(), tr.cpu().numpy(), acts.cpu().numpy()
    s = init.copy()
    c = np.zeros(B, np.int32)
    for t in range(K):
        r, d_, t_, e, _, _ = O.env_step(s, A[t], L, H, c, reset_state=init)
        assert not e.any()
        assert np.array_equal(R[t], r), t
        assert np.array_equal(D[t], d_) and np.array_equal(T[t], t_), t
        assert np.array_equal(obs_s[t], s[sample]), t
    assert T[K - 1].sum() > B // 2  # the horizon ends on the last step for every env that never finished
    assert np.array_equal(state.cpu().numpy(), s) and np.array_equal(cnt.cpu().numpy(), c)
    assert int(ec.item()) == 0


@pytest.mark.parametrize("L", [128, 36])
def test_config5_shard_every_env_vs_oracle(L):
    """BASELINE configs[4]'s per-GPU shard (2^20 envs, L = 128, Miller-Schupp starts, random moves,
    horizon 200) through VecACEnv.step -- acx_step_lengths_reduced once the rows' lengths are
    current (lengths and reduced flags carried) -- on every env and step against the C oracle:
    states, rewards, flags and the carried lengths.  L = 36: the same batch at configs[2]'s L,
    which VecACEnv also steps with the reduced lengths-carrying kernel (ops.lengths_step_for)."""
    import bench
    from acx import VecACEnv, ops
    B, K, H = 1 << 20, 8, 200
    assert ops.lengths_step_for(B, L)
    init = bench.ms_starts(L, B)
    env = VecACEnv(init, horizon_length=H, device=DEV, track_final_obs=False)
    g = torch.Generator(device=DEV)
    g.manual_seed(5)
    s = init.copy()
    c = np.zeros(B, np.int32)
    for t in range(K):
        a = torch.randint(0, 12, (B,), dtype=torch.int32, device=DEV, generator=g)
        st, rew, dn, tr, _ = env.step(a)
        r, d_, t_, e, lens, _ = O.env_step(s, a.cpu().numpy(), L, H, c, reset_state=init)
        assert not e.any()
        assert np.array_equal(st.cpu().numpy(), s), t
        assert np.array_equal(rew.cpu().numpy(), r), t
        assert np.array_equal(dn.cpu().numpy(), d_) and np.array_equal(tr.cpu().numpy(), t_), t
        assert np.array_equal(env.lengths.cpu().numpy(), lens), t
    assert np.array_equal(env.step_count.cpu().numpy(), c)
    # every row that moved is known reduced; a row that ended (solved: done) restarted from its
    # starting row and is read whole next time
    fin = (dn | tr).bool()
    assert torch.equal(env.reduced != 0, ~fin) and int(fin.sum().item()) < B // 100


def test_config2_full_horizon_every_env_vs_oracle():
    """BASELINE configs[1] as bench.py's config2_step runs it: 65,536 Miller-Schupp starts, L = 36,
    horizon 200, 200 per-call in-place steps through ops.StepPlan (the small-batch step kernel),
    through one synchronised truncation -- every env and step against the C oracle."""
    import bench
    from acx import ops
    L, B, K, H = 36, 65536, 200, 200
    init = bench.ms_starts(L, B)
    starts = torch.as_tensor(init).to(DEV)
    st = starts.clone()
    cnt = torch.zeros(B, dtype=torch.int32, device=DEV)
    rew = torch.empty(B, dtype=torch.int32, device=DEV)
    dn = torch.empty(B, dtype=torch.uint8, device=DEV)
    tr = torch.empty(B, dtype=torch.uint8, device=DEV)
    lens = torch.empty((B, 2), dtype=torch.int32, device=DEV)
    err = torch.zeros(B, dtype=torch.uint8, device=DEV)
    step = ops.StepPlan(st, state_out=st, reset_state=starts, step_count=cnt, horizon=H, cyclical=True, reward=rew,
                        done=dn, truncated=tr, lengths=lens, err=err)
    g = torch.Generator(device=DEV)
    g.manual_seed(0)
    acts = torch.randint(0, 12, (K, B), dtype=torch.int32, device=DEV, generator=g)
    A = acts.cpu().numpy()
    s = init.copy()
    c = np.zeros(B, np.int32)
    n_trunc = 0
    for t in range(K):
        step(acts[t])
        r, d_, t_, e, ln, _ = O.env_step(s, A[t], L, H, c, reset_state=init)
        assert not e.any()
        assert np.array_equal(st.cpu().numpy(), s), t
        assert np.array_equal(rew.cpu().numpy(), r) and np.array_equal(dn.cpu().numpy(), d_), t
        assert np.array_equal(tr.cpu().numpy(), t_) and np.array_equal(lens.cpu().numpy(), ln), t
        n_trunc += int(t_.sum())
    assert n_trunc > B // 2  # the horizon's synchronised truncation was stepped through
