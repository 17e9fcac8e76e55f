"""GPU: the lengths-carrying step (acx_step_lengths: in place, the rows' relator lengths in and
out, only the chunks inside the letters read and written) against acx_step on the same rows,
actions and starting states, many steps: states, rewards, flags, step counts, final
observations, errors and lengths bit-exact.  acx_step is itself pinned to the reference's
fixtures (test_gpu_parity.py), and the full-size in-place test there runs the lengths-carrying
stream beside it at 2^20 envs.  VecACEnv's plain step takes acx_step_lengths at L = 128
(ops.LENGTHS_STEP_L)."""
import numpy as np
import pytest
import torch

from conftest import REPO  # noqa: F401

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


def _rows(L, B, rng):
    """canonical rows of mixed lengths (0 .. L letters per relator), a tenth trivial"""
    s = np.zeros((B, 2 * L), np.int32)
    letters = np.array([1, -1, 2, -2], np.int32)
    for b in range(B):
        for h in range(2):
            n = int(rng.integers(1, L + 1)) if b % 10 else 1
            w = []
            while len(w) < n:  # freely reduced
                x = int(letters[rng.integers(0, 4)])
                if w and w[-1] == -x:
                    continue
                w.append(x)
            if b % 10 == 0:
                w = [1 + h]
            s[b, h * L:h * L + n] = w
    return s


def _t(x):
    return torch.as_tensor(np.ascontiguousarray(x)).to(DEV)


def _check_reduced_flags(flags, rows, L, where):
    """acx_step_lengths_reduced's flags claim only what holds: bit 0 -> both relators non-empty and
    freely reduced, bit 1 -> and cyclically reduced (include/acx.h)"""
    f = flags.cpu().numpy()
    s = rows.cpu().numpy() if torch.is_tensor(rows) else rows
    assert ((f & ~np.uint8(3)) == 0).all(), where
    assert not ((f & 2) & ~((f & 1) << 1)).any(), where  # cyclically reduced implies freely
    for b in np.flatnonzero(f):
        for h in range(2):
            w = s[b, h * L:(h + 1) * L]
            n = int(np.count_nonzero(w))
            assert n > 0 and not w[n:].any() and (w[:n] != 0).all(), (where, b, h)
            assert not (w[1:n] == -w[: n - 1]).any(), (where, b, h)
            if f[b] & 2 and n > 1:
                assert w[0] != -w[n - 1], (where, b, h)
    return int((f != 0).sum())


@pytest.mark.parametrize("L", [36, 128, 18, 64])
@pytest.mark.parametrize("cyc", [0, 1])
@pytest.mark.parametrize("reduced", [False, True])
def test_step_lengths_matches_acx_step(L, cyc, reduced):
    """reduced: acx_step_lengths_reduced, the reduced flags carried from call to call (a
    conjugation of a reduced row leaves its other relator unread)"""
    from acx import _lib
    lib = _lib.load()
    rng = np.random.default_rng(L * 7 + cyc)
    B, T, H = 64 * 37 + 11, 40, 9
    start = _rows(L, B, rng)
    reset = _rows(L, B, rng)
    reset[5::97, 3] = 3  # out-of-domain starting rows: envs that reset onto them become ACX_ERR_DOMAIN
    n_ood = len(range(5, B, 97))
    st = {k: _t(start) for k in "ab"}
    rs = _t(reset)
    cnt = {k: torch.zeros(B, dtype=torch.int32, device=DEV) for k in "ab"}
    rew = {k: torch.zeros(B, dtype=torch.int32, device=DEV) for k in "ab"}
    dn = {k: torch.zeros(B, dtype=torch.uint8, device=DEV) for k in "ab"}
    tr = {k: torch.zeros(B, dtype=torch.uint8, device=DEV) for k in "ab"}
    fo = {k: torch.zeros((B, 2 * L), dtype=torch.int32, device=DEV) for k in "ab"}
    err = {k: torch.zeros(B, dtype=torch.uint8, device=DEV) for k in "ab"}
    ec = {k: torch.zeros(1, dtype=torch.int32, device=DEV) for k in "ab"}
    lens_a = torch.zeros((B, 2), dtype=torch.int32, device=DEV)
    lens_b = _t(np.stack([np.count_nonzero(start[:, :L], 1), np.count_nonzero(start[:, L:], 1)], 1).astype(np.int32))
    lens_b[::13] = L  # (L, L): "read the whole row", always safe
    red = torch.zeros(B, dtype=torch.uint8, device=DEV)
    stream = torch.cuda.current_stream(DEV).cuda_stream
    n_reset = n_err = n_flagged = 0
    for t in range(T):
        a = rng.integers(0, 12, size=B).astype(np.int32)
        if t % 7 == 3:
            a[::211] = 12  # ACX_ERR_ACTION: the row is left as it is
        at = _t(a)
        for k in "ab":
            P = lambda x: x[k].data_ptr()  # noqa: E731
            if k == "a":
                rc = lib.acx_step(P(st), P(st), at.data_ptr(), rs.data_ptr(), P(cnt), P(rew), P(dn), P(tr),
                                  lens_a.data_ptr(), P(fo), P(err), P(ec), B, L, H, cyc, stream)
            elif reduced:
                rc = lib.acx_step_lengths_reduced(P(st), at.data_ptr(), rs.data_ptr(), P(cnt), P(rew), P(dn),
                                                  P(tr), lens_b.data_ptr(), red.data_ptr(), P(fo), P(err), P(ec),
                                                  B, L, H, cyc, stream)
            else:
                rc = lib.acx_step_lengths(P(st), at.data_ptr(), rs.data_ptr(), P(cnt), P(rew), P(dn), P(tr),
                                          lens_b.data_ptr(), P(fo), P(err), P(ec), B, L, H, cyc, stream)
            assert rc == 0, (k, rc)
        for name, d in (("state", st), ("reward", rew), ("done", dn), ("trunc", tr), ("count", cnt),
                        ("final_obs", fo), ("err", err), ("err_count", ec)):
            assert torch.equal(d["a"], d["b"]), (t, name)
        if reduced:
            n_flagged += _check_reduced_flags(red, st["b"], L, t)
        e = err["a"].cpu().numpy()
        dom = e == 3
        la, lb = lens_a.cpu().numpy(), lens_b.cpu().numpy()
        assert np.array_equal(la[~dom], lb[~dom]), t
        assert (lb[dom] == L).all(), t  # out-of-domain rows are read whole on the next call
        # the lengths are the rows' own (canonical rows: letters, then zero padding)
        s = st["b"].cpu().numpy()
        ok = ~dom
        assert np.array_equal(lb[ok, 0], np.count_nonzero(s[ok, :L], 1)), t
        assert np.array_equal(lb[ok, 1], np.count_nonzero(s[ok, L:], 1)), t
        n_reset += int((dn["a"] | tr["a"]).sum())
        n_err += int((e != 0).sum())
    assert n_reset > B and n_err > n_ood  # resets, out-of-domain resets and failed moves exercised
    if reduced:
        assert n_flagged > T * B // 2  # most rows stepped as known-reduced


@pytest.mark.parametrize("L", [36, 128, 17])
@pytest.mark.parametrize("reduced", [False, True])
def test_step_lengths_error_stream_matches_acx_step(L, reduced):
    """The error-contract stream of test_gpu_rollout_errors (moves that empty a relator from
    r0 == r1 rows, an unreduced relator whose conjugation raises, out-of-domain INPUT rows -- a
    letter 3, a zero inside r1, a letter 300 -- and out-of-domain starting rows, bad move ids,
    desynchronised and whole-wave resets) through acx_step_lengths with the lengths VecACEnv
    computes (_row_extent: far enough to see every bad entry), against acx_step."""
    from test_gpu_rollout_errors import _error_stream
    from acx import _lib
    from acx.envs.ac_env import _row_extent
    lib = _lib.load()
    B, T, H = 64 * 11 + 21, 26, 6
    st0, resets, count0, acts, eq, bad_in, bad_rs = _error_stream(L, B, T, H, seed=L + 7)
    st = {k: _t(st0) for k in "ab"}
    rs = _t(resets)
    cnt = {k: _t(count0) for k in "ab"}
    rew = {k: torch.zeros(B, dtype=torch.int32, device=DEV) for k in "ab"}
    dn = {k: torch.zeros(B, dtype=torch.uint8, device=DEV) for k in "ab"}
    tr = {k: torch.zeros(B, dtype=torch.uint8, device=DEV) for k in "ab"}
    err = {k: torch.zeros(B, dtype=torch.uint8, device=DEV) for k in "ab"}
    ec = {k: torch.zeros(1, dtype=torch.int32, device=DEV) for k in "ab"}
    lens_a = torch.zeros((B, 2), dtype=torch.int32, device=DEV)
    lens_b = _row_extent(st["b"], L).contiguous()
    red = torch.zeros(B, dtype=torch.uint8, device=DEV)
    stream = torch.cuda.current_stream(DEV).cuda_stream
    seen = set()
    for t in range(T):
        at = _t(acts[t])
        for k in "ab":
            P = lambda x: x[k].data_ptr()  # noqa: E731
            if k == "a":
                rc = lib.acx_step(P(st), P(st), at.data_ptr(), rs.data_ptr(), P(cnt), P(rew), P(dn), P(tr),
                                  lens_a.data_ptr(), None, P(err), P(ec), B, L, H, 1, stream)
            elif reduced:
                rc = lib.acx_step_lengths_reduced(P(st), at.data_ptr(), rs.data_ptr(), P(cnt), P(rew), P(dn),
                                                  P(tr), lens_b.data_ptr(), red.data_ptr(), None, P(err), P(ec),
                                                  B, L, H, 1, stream)
            else:
                rc = lib.acx_step_lengths(P(st), at.data_ptr(), rs.data_ptr(), P(cnt), P(rew), P(dn), P(tr),
                                          lens_b.data_ptr(), None, P(err), P(ec), B, L, H, 1, stream)
            assert rc == 0, (k, rc)
        for name, d in (("state", st), ("reward", rew), ("done", dn), ("trunc", tr), ("count", cnt),
                        ("err", err), ("err_count", ec)):
            assert torch.equal(d["a"], d["b"]), (t, name)
        if reduced:
            _check_reduced_flags(red, st["b"], L, t)
        e = err["a"].cpu().numpy()
        dom = e == 3
        la, lb = lens_a.cpu().numpy(), lens_b.cpu().numpy()
        assert np.array_equal(la[~dom], lb[~dom]), t
        assert (lb[dom] == L).all(), t
        seen |= set(np.unique(e).tolist())
    assert {1, 2, 3, 4} <= seen  # every error kind went through both calls


def test_step_lengths_rejects_missing_lengths():
    from acx import _lib
    lib = _lib.load()
    L, B = 36, 64
    s = _t(_rows(L, B, np.random.default_rng(0)))
    a = torch.zeros(B, dtype=torch.int32, device=DEV)
    stream = torch.cuda.current_stream(DEV).cuda_stream
    rc = lib.acx_step_lengths(s.data_ptr(), a.data_ptr(), None, None, None, None, None, None, None, None, None,
                              B, L, 5, 1, stream)
    assert rc == _lib.E_ARG
    ln = torch.full((B, 2), L, dtype=torch.int32, device=DEV)
    rc = lib.acx_step_lengths_reduced(s.data_ptr(), a.data_ptr(), None, None, None, None, None, ln.data_ptr(), None,
                                      None, None, None, B, L, 5, 1, stream)
    assert rc == _lib.E_ARG  # the reduced flags are required


@pytest.mark.parametrize("L", [128, 36])
def test_vec_env_lengths_after_rollout_and_direct_writes(L):
    """VecACEnv keeps lengths current across steps; a rollout (no lengths out) and reset_env
    hand over correctly: the env matches a twin stepped one move at a time with acx_step.  At
    L = 128 the env's steps go through acx_step_lengths (ops.LENGTHS_STEP_L)."""
    from acx import VecACEnv, _lib, ops
    B, H = 64 * 5 + 3, 8
    rng = np.random.default_rng(3)
    start = _rows(L, B, rng)
    env = VecACEnv(start, horizon_length=H, device=DEV)
    assert env._live_tile == ops.lengths_step_for(B, L)
    twin = VecACEnv(start, horizon_length=H, device=DEV)
    twin._lengths_ok = False  # the twin always takes acx_step (it rewrites its lengths each call)
    T = 6
    acts = rng.integers(0, 12, size=(T + 4, B)).astype(np.int32)
    env.rollout(_t(acts[:T]))
    assert not env._lengths_ok
    for t in range(T):
        twin.step(_t(acts[t]))
        twin._lengths_ok = False
    assert torch.equal(env.state, twin.state)
    new = _rows(L, 1, rng)[0]
    env.reset_env(7, new)
    twin.reset_env(7, new)
    for t in range(T, T + 4):
        o1, r1, d1, t1, _ = env.step(_t(acts[t]))
        assert env._lengths_ok
        o2, r2, d2, t2, _ = twin.step(_t(acts[t]))
        twin._lengths_ok = False
        for x, y in ((o1, o2), (r1, r2), (d1, d2), (t1, t2), (env.step_count, twin.step_count)):
            assert torch.equal(x, y), t
        assert torch.equal(env.lengths, twin.lengths), t
    assert _lib.E_ARG < 0


# ---------------------------------------------------------------------------------------------
# acx_step_lengths pinned directly to the reference fixtures and to the oracle (VERDICT r04
# item 3): the reference's carried lengths are ac_env.py:81-95 (self.lengths from reset, passed to
# and returned by ACMove) and ac_moves.py:159-231.
# ---------------------------------------------------------------------------------------------
def _lengths_step(lib, st, at, rs, cnt, rew, dn, tr, lens, fo, err, ec, B, L, H, cyc, red=None):
    stream = torch.cuda.current_stream(DEV).cuda_stream
    P = lambda x: None if x is None else x.data_ptr()  # noqa: E731
    if red is not None:
        rc = lib.acx_step_lengths_reduced(P(st), P(at), P(rs), P(cnt), P(rew), P(dn), P(tr), P(lens), P(red), P(fo),
                                          P(err), P(ec), B, L, H, cyc, stream)
    else:
        rc = lib.acx_step_lengths(P(st), P(at), P(rs), P(cnt), P(rew), P(dn), P(tr), P(lens), P(fo), P(err), P(ec),
                                  B, L, H, cyc, stream)
    assert rc == 0, rc


@pytest.mark.parametrize("L", [7, 18, 36, 128])
@pytest.mark.parametrize("cyc", [1, 0])
def test_step_lengths_transitions_fixture(L, cyc):
    """The reference's random transitions (tests/golden/transitions.npz, made by running the
    reference's ACMove): in place, with the lengths VecACEnv carries in (_row_extent); every
    row ends as the reference's output with the reference's lengths, failed rows keep their input
    row (and report (L, L) when out of domain, so the next call reads them whole)."""
    from acx import _lib
    from acx.envs.ac_env import _row_extent
    from conftest import GOLDEN
    import os
    lib = _lib.load()
    d = np.load(os.path.join(GOLDEN, "transitions.npz"))
    k = f"L{L}_c{cyc}_"
    s_in = d[k + "state_in"].astype(np.int32)
    B = s_in.shape[0]
    st = _t(s_in)
    lens = _row_extent(st, L).contiguous()
    err = torch.zeros(B, dtype=torch.uint8, device=DEV)
    _lengths_step(lib, st, _t(d[k + "action"].astype(np.int32)), None, None, None, None, None, lens, None, err,
                  None, B, L, 10 ** 6, cyc)
    out, e, ln = st.cpu().numpy(), err.cpu().numpy(), lens.cpu().numpy()
    assert np.array_equal(e, d[k + "err"].astype(np.uint8))
    ok = e == 0
    assert ok.sum() > B // 2
    assert np.array_equal(out[ok], d[k + "state_out"][ok].astype(np.int32))
    assert np.array_equal(ln[ok], d[k + "lengths"][ok].astype(np.int32))
    assert np.array_equal(out[~ok], s_in[~ok])
    assert (ln[e == 3] == L).all()


def test_step_lengths_reference_episodes():
    """ACEnv episodes run by the reference (tests/golden/env_episodes.npz, explicit reset() on done
    or truncated): acx_step_lengths with same-step autoreset reproduces every step's observation,
    reward, flags and final observation, and its carried lengths stay the rows' letter counts."""
    from acx import _lib
    from conftest import GOLDEN
    import os
    lib = _lib.load()
    d = np.load(os.path.join(GOLDEN, "env_episodes.npz"))
    L, H = int(d["L"]), int(d["horizon"])
    init = d["initial"].astype(np.int32)
    B = init.shape[0]
    st, rs = _t(init), _t(init)
    lens = _t(np.stack([np.count_nonzero(init[:, :L], 1), np.count_nonzero(init[:, L:], 1)], 1).astype(np.int32))
    cnt = torch.zeros(B, dtype=torch.int32, device=DEV)
    rew = torch.zeros(B, dtype=torch.int32, device=DEV)
    dn = torch.zeros(B, dtype=torch.uint8, device=DEV)
    tr = torch.zeros(B, dtype=torch.uint8, device=DEV)
    fo = torch.zeros((B, 2 * L), dtype=torch.int32, device=DEV)
    err = torch.zeros(B, dtype=torch.uint8, device=DEV)
    ec = torch.zeros(1, dtype=torch.int32, device=DEV)
    for t in range(d["actions"].shape[0]):
        _lengths_step(lib, st, _t(d["actions"][t].astype(np.int32)), rs, cnt, rew, dn, tr, lens, fo, err, ec, B, L,
                      H, 1)
        obs = st.cpu().numpy()
        assert np.array_equal(obs, d["obs"][t].astype(np.int32)), t
        assert np.array_equal(rew.cpu().numpy(), d["reward"][t]), t
        assert np.array_equal(dn.cpu().numpy(), d["done"][t].astype(np.uint8)), t
        assert np.array_equal(tr.cpu().numpy(), d["truncated"][t].astype(np.uint8)), t
        m = (d["done"][t] | d["truncated"][t]).astype(bool)
        assert np.array_equal(fo.cpu().numpy()[m], d["final_obs"][t][m].astype(np.int32)), t
        ln = lens.cpu().numpy()
        assert np.array_equal(ln[:, 0], np.count_nonzero(obs[:, :L], 1)), t
        assert np.array_equal(ln[:, 1], np.count_nonzero(obs[:, L:], 1)), t
    assert int(ec.item()) == 0


@pytest.mark.parametrize("cyc", [1, 0])
@pytest.mark.parametrize("reduced", [False, True])
def test_step_lengths_walk_with_resets_vs_oracle_L128(cyc, reduced):
    """A random walk at L = 128 (config 5's kernel) with autoreset -- short horizon, desynchronised
    and synchronised resets, a few bad move ids -- every env, every step against the oracle's
    ACMove (oracle/acx_oracle.c, pinned to the reference's fixtures) under acx's error contract
    (conftest.env_step_contract: a failed move keeps state and count): state, reward, done,
    truncated, step count, err, final observation and the carried lengths."""
    from acx import _lib
    from conftest import env_step_contract
    from oracle import oracle as O
    lib = _lib.load()
    L, B, T, H = 128, 64 * 23 + 5, 60, 13
    rng = np.random.default_rng(128 + cyc)
    starts = _rows(L, B, rng)
    count0 = (np.arange(B) % H).astype(np.int32)
    count0[: 64 * 4] = 0  # four whole waves truncate together (the tile-reload path)
    st, rs = _t(starts), _t(starts)
    cnt = _t(count0)
    lens = _t(np.stack([np.count_nonzero(starts[:, :L], 1), np.count_nonzero(starts[:, L:], 1)], 1).astype(np.int32))
    rew = torch.zeros(B, dtype=torch.int32, device=DEV)
    dn = torch.zeros(B, dtype=torch.uint8, device=DEV)
    tr = torch.zeros(B, dtype=torch.uint8, device=DEV)
    fo = torch.zeros((B, 2 * L), dtype=torch.int32, device=DEV)
    err = torch.zeros(B, dtype=torch.uint8, device=DEV)
    red = torch.zeros(B, dtype=torch.uint8, device=DEV) if reduced else None
    o_st, o_cnt = starts.copy(), count0.copy()
    n_reset = n_err = 0
    for t in range(T):
        a = rng.integers(0, 12, size=B).astype(np.int32)
        if t % 11 == 5:
            a[::97] = -1  # ACX_ERR_ACTION: state and count kept
        _lengths_step(lib, st, _t(a), rs, cnt, rew, dn, tr, lens, fo, err, None, B, L, H, cyc, red)
        # the pre-reset states (final_observation), then the step under acx's error contract (a
        # failed move keeps state and count: conftest.env_step_contract, checked against the oracle)
        moved, _, merr = O.move_batch(o_st, a, L, cyc)
        fin = o_st.copy()
        fin[merr == 0] = moved[merr == 0]
        r, d_, trn, e = env_step_contract(o_st, a, o_cnt, starts, L, H, cyc)
        assert np.array_equal(st.cpu().numpy(), o_st), t
        assert np.array_equal(err.cpu().numpy(), e), t
        ok = e == 0
        assert np.array_equal(rew.cpu().numpy(), r), t
        assert np.array_equal(dn.cpu().numpy(), d_), t
        assert np.array_equal(tr.cpu().numpy(), trn), t
        assert np.array_equal(cnt.cpu().numpy(), o_cnt), t
        m = (d_ | trn).astype(bool)
        assert np.array_equal(fo.cpu().numpy()[m], fin[m]), t
        got = lens.cpu().numpy()
        assert np.array_equal(got[:, 0], np.count_nonzero(o_st[:, :L], 1)), t
        assert np.array_equal(got[:, 1], np.count_nonzero(o_st[:, L:], 1)), t
        n_reset += int(m.sum())
        n_err += int((~ok).sum())
        if reduced:
            _check_reduced_flags(red, o_st, L, t)
    assert n_reset > B and n_err > 0


@pytest.mark.parametrize("L", [128, 36])
def test_step_lengths_reduced_flags_across_cyclical_modes(L):
    """The reduced flags carried through calls that alternate cyclical=True / False (bit 1 set only
    by cyclical calls, bit 0 by both): every call equals acx_step on the same rows, and a flagged
    row is reduced in the sense its bits claim."""
    from acx import _lib
    lib = _lib.load()
    rng = np.random.default_rng(L + 99)
    B, T, H = 64 * 19 + 7, 24, 11
    start = _rows(L, B, rng)
    st = {k: _t(start) for k in "ab"}
    rs = _t(start)
    cnt = {k: torch.zeros(B, dtype=torch.int32, device=DEV) for k in "ab"}
    rew = {k: torch.zeros(B, dtype=torch.int32, device=DEV) for k in "ab"}
    dn = {k: torch.zeros(B, dtype=torch.uint8, device=DEV) for k in "ab"}
    tr = {k: torch.zeros(B, dtype=torch.uint8, device=DEV) for k in "ab"}
    err = {k: torch.zeros(B, dtype=torch.uint8, device=DEV) for k in "ab"}
    lens_a = torch.zeros((B, 2), dtype=torch.int32, device=DEV)
    lens_b = _t(np.stack([np.count_nonzero(start[:, :L], 1), np.count_nonzero(start[:, L:], 1)], 1).astype(np.int32))
    red = torch.zeros(B, dtype=torch.uint8, device=DEV)
    stream = torch.cuda.current_stream(DEV).cuda_stream
    seen = set()
    for t in range(T):
        cyc = (t // 3) % 2  # three steps in each mode
        at = _t(rng.integers(0, 12, size=B).astype(np.int32))
        P = lambda x, k: x[k].data_ptr()  # noqa: E731
        assert lib.acx_step(P(st, "a"), P(st, "a"), at.data_ptr(), rs.data_ptr(), P(cnt, "a"), P(rew, "a"),
                            P(dn, "a"), P(tr, "a"), lens_a.data_ptr(), None, P(err, "a"), None, B, L, H, cyc,
                            stream) == 0
        assert lib.acx_step_lengths_reduced(P(st, "b"), at.data_ptr(), rs.data_ptr(), P(cnt, "b"), P(rew, "b"),
                                            P(dn, "b"), P(tr, "b"), lens_b.data_ptr(), red.data_ptr(), None,
                                            P(err, "b"), None, B, L, H, cyc, stream) == 0
        for name, d in (("state", st), ("reward", rew), ("done", dn), ("trunc", tr), ("count", cnt), ("err", err)):
            assert torch.equal(d["a"], d["b"]), (t, name)
        _check_reduced_flags(red, st["b"], L, t)
        seen |= set(np.unique(red.cpu().numpy()).tolist())
    assert {0, 1, 3} <= seen  # both modes' flags and unflagged (reset) rows occurred
