"""GPU parity of the exact int32-letter word kernels (csrc/acx_words.hip) and of the
reference-signature wrappers built on them (acx.envs.ac_moves / acx.envs.utils):
  * the reference's own unit cases (tests/test_ac_env.py:17-538 re-run by make_golden.py,
    letters 3..6 included), through concatenate_relators / conjugate / simplify_relator /
    simplify_presentation / ACMove exactly as the reference's tests call them;
  * every small-L reference transition (smallL_random.npz: unreduced words, empty relators,
    zeros inside relators, every error kind) through acx_word_move;
  * random generic-letter inputs (letters up to +-6, zeros inside relators, long relator arrays)
    against the oracle, which is pinned to the reference on CPU (tests/test_oracle.py);
  * ACEnv episodes on presentations with letters beyond +-2."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import oracle as O

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


@pytest.fixture(scope="module")
def unit():
    with open(os.path.join(GOLDEN, "unit_cases.json")) as f:
        return json.load(f)


def test_reference_unit_cases_through_acx(unit):
    from acx.envs import ac_moves as M
    from acx.envs import utils as U
    for c in unit["simplify_relator"]:  # tests/test_ac_env.py:17-83
        r, n = U.simplify_relator(np.array(c["relator"]), c["L"], cyclical=c["cyclical"], padded=c["padded"])
        assert r.tolist() == c["out"] and n == c["n"], c
    for c in unit["simplify_presentation"]:  # :140-181
        o, lens = U.simplify_presentation(np.array(c["p"]), c["L"], [0, 0], cyclical=c["cyclical"])
        assert o.tolist() == c["out"] and lens == c["lengths"], c
    for c in unit["concatenate"]:  # :184-326
        p = np.array(c["p"])
        lens = [int(np.count_nonzero(p[: c["L"]])), int(np.count_nonzero(p[c["L"]:]))]
        o, ol = M.concatenate_relators(p, c["L"], c["i"], c["j"], c["sign"], lens)
        assert o.tolist() == c["out"] and ol == c["lengths"], c
    for c in unit["conjugate"]:  # :329-477
        p = np.array(c["p"])
        lens = [int(np.count_nonzero(p[: c["L"]])), int(np.count_nonzero(p[c["L"]:]))]
        o, ol = M.conjugate(p, c["L"], c["i"], c["j"], c["sign"], lens)
        assert o.tolist() == c["out"] and ol == c["lengths"], c
    for c in unit["acmove"]:  # :495-538, all 12 moves, both flags, letters 3..6
        p = np.array(c["p"])
        if c["raises"]:
            with pytest.raises({"AssertionError": AssertionError, "IndexError": IndexError}[c["raises"]]):
                M.ACMove(c["move"], p, c["L"], [0, 0], cyclical=c["cyclical"])
            continue
        o, ol = M.ACMove(c["move"], p, c["L"], [0, 0], cyclical=c["cyclical"])
        assert o.tolist() == c["out"] and ol == c["lengths"], c


def test_small_L_reference_transitions_through_word_kernel():
    from acx import ops
    d = np.load(os.path.join(GOLDEN, "smallL_random.npz"))
    for L in range(1, 10):
        S = d[f"L{L}_state_in"].astype(np.int32)
        A = d[f"L{L}_action"].astype(np.int32)
        C = d[f"L{L}_cyclical"]
        for cyc in (0, 1):
            sel = C == cyc
            st = torch.as_tensor(S[sel]).to(DEV)
            out, lens, done, err = ops.word_move(st, torch.as_tensor(A[sel]).to(DEV), cyclical=bool(cyc))
            e = err.cpu().numpy()
            want_e = d[f"L{L}_err"][sel]
            assert np.array_equal(e, want_e), L
            ok = want_e == 0
            assert np.array_equal(out.cpu().numpy()[ok], d[f"L{L}_state_out"][sel][ok].astype(np.int32)), L
            assert np.array_equal(lens.cpu().numpy()[ok], d[f"L{L}_lengths"][sel][ok]), L
            # rows that raise keep their input
            assert np.array_equal(out.cpu().numpy()[~ok], S[sel][~ok]), L


def _random_generic(rng, B, L, zero_frac=0.05, letters=6):
    s = np.zeros((B, 2 * L), np.int32)
    for b in range(B):
        for h in range(2):
            n = 0 if rng.random() < 0.04 else int(rng.integers(1, L + 1))
            s[b, h * L : h * L + n] = rng.choice([k for k in range(-letters, letters + 1) if k], size=n)
        if rng.random() < zero_frac:
            s[b, int(rng.integers(2 * L))] = 0
    return s


@pytest.mark.parametrize("L", [1, 2, 5, 7, 36, 128])
@pytest.mark.parametrize("cyc", [True, False])
def test_word_move_generic_letters_equal_oracle(L, cyc):
    from acx import ops
    rng = np.random.default_rng(L * 7 + cyc)
    B = 3000 if L < 100 else 500
    s = _random_generic(rng, B, L)
    a = rng.integers(-1, 13, size=B).astype(np.int32)
    out, lens, done, err = ops.word_move(torch.as_tensor(s).to(DEV), torch.as_tensor(a).to(DEV), cyclical=cyc)
    out, lens, done, err = (x.cpu().numpy() for x in (out, lens, done, err))
    for b in range(B):
        o, ln, e = O.move(s[b], L, a[b], cyc)
        assert err[b] == e, (b, s[b], a[b])
        assert np.array_equal(out[b], o) and list(lens[b]) == ln, (b, s[b], a[b])
        assert done[b] == (e == 0 and sum(ln) == 2 and O.is_trivial(o)), b


@pytest.mark.parametrize("L", [3, 36, 128])
def test_concatenate_conjugate_generic_equal_oracle(L):
    from acx import ops
    rng = np.random.default_rng(L)
    B = 2000 if L < 100 else 400
    s = _random_generic(rng, B, L)
    st = torch.as_tensor(s).to(DEV)
    for i in (0, 1):
        for sign in (1, -1):
            out, lo = ops.concatenate(st, i, 1 - i, sign)
            out, lo = out.cpu().numpy(), lo.cpu().numpy()
            for b in range(B):
                assert np.array_equal(out[b], O.concatenate(s[b], L, i, 1 - i, sign)), (b, i, sign)
            for j in (1, 2):
                out, lo, err = ops.conjugate(st, i, j, sign)
                out, err = out.cpu().numpy(), err.cpu().numpy()
                for b in range(B):
                    o, e = O.conjugate(s[b], L, i, j, sign)
                    assert err[b] == e, (b, i, j, sign)
                    assert np.array_equal(out[b], o if e == 0 else s[b]), (b, i, j, sign)


@pytest.mark.parametrize("m,L", [(5, 5), (9, 4), (4, 9), (40, 36), (130, 128), (1, 1)])
@pytest.mark.parametrize("cyc", [True, False])
@pytest.mark.parametrize("padded", [True, False])
def test_simplify_relator_generic_equal_oracle(m, L, cyc, padded):
    from acx import ops
    rng = np.random.default_rng(m * 31 + L)
    B = 1000
    rel = np.zeros((B, m), np.int32)
    for b in range(B):
        n = int(rng.integers(0, m + 1))
        rel[b, :n] = rng.choice([-3, -2, -1, 1, 2, 3], size=n)
        if rng.random() < 0.05 and m > 1:
            rel[b, int(rng.integers(m))] = 0
    out, ol, n, err = ops.word_simplify_relator(torch.as_tensor(rel).to(DEV), L, cyclical=cyc, padded=padded)
    out, ol, n, err = (x.cpu().numpy() for x in (out, ol, n, err))
    for b in range(B):
        o, nn, e = O.simplify_relator(rel[b], L, cyc, padded)
        assert err[b] == e, (b, rel[b])
        if e == 0:
            assert out[b, : ol[b]].tolist() == o.tolist() and n[b] == nn, (b, rel[b])


def test_acenv_with_generic_letters_equals_oracle():
    """ACEnvConfig accepts any integer letters (it validates the zero padding only,
    ac_env.py:22-35 -> utils.py:13-54); ACEnv then steps through the exact word kernel."""
    import acx
    rng = np.random.default_rng(3)
    L, H = 6, 9
    for k in range(6):
        s = _random_generic(rng, 1, L, zero_frac=0.0, letters=4)[0]
        s[0], s[L] = 3, -4  # non-empty relators with letters beyond +-2
        env = acx.ACEnv(acx.ACEnvConfig(initial_state=s.astype(np.int64), horizon_length=H))
        o_state = s.copy()
        cnt = 0
        for t in range(25):
            a = int(rng.integers(12))
            o, ln, e = O.move(o_state, L, a, True)
            if e:
                with pytest.raises((AssertionError, IndexError)):
                    env.step(a)
                break
            st, r, d, tr, info = env.step(a)
            o_state = o
            cnt += 1
            od = sum(ln) == 2 and O.is_trivial(o)
            assert st.tolist() == o.tolist() and env.lengths == ln
            assert d == od and r == (H * L * 2 if od else -sum(ln)) and tr == (cnt >= H)
            if d or tr:
                env.reset()
                o_state = s.copy()
                cnt = 0
