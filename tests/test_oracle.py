"""Pin the CPU oracle (oracle/acx_oracle.c) against fixtures produced by the reference
itself (tests/golden/make_golden.py).  CPU only."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import oracle as O


def _load(name):
    return np.load(os.path.join(GOLDEN, name))


@pytest.fixture(scope="module")
def unit():
    with open(os.path.join(GOLDEN, "unit_cases.json")) as f:
        return json.load(f)


def test_simplify_relator_cases(unit):
    # tests/test_ac_env.py:17-83
    for c in unit["simplify_relator"]:
        out, n, e = O.simplify_relator(c["relator"], c["L"], c["cyclical"], c["padded"])
        assert e == 0
        assert out.tolist() == c["out"], c
        assert n == c["n"]


def test_valid_and_trivial_cases(unit):
    for c in unit["valid"]:
        assert O.is_valid(c["p"]) == c["out"], c
    for c in unit["trivial"]:
        assert O.is_trivial(c["p"]) == c["out"], c


def test_simplify_presentation_cases(unit):
    for c in unit["simplify_presentation"]:
        out, lens, e = O.simplify_presentation(c["p"], c["L"], c["cyclical"])
        assert e == 0
        assert out.tolist() == c["out"] and lens == c["lengths"], c


def test_concatenate_conjugate_cases(unit):
    for c in unit["concatenate"]:
        out = O.concatenate(c["p"], c["L"], c["i"], c["j"], c["sign"])
        assert out.tolist() == c["out"], c
    for c in unit["conjugate"]:
        out, e = O.conjugate(c["p"], c["L"], c["i"], c["j"], c["sign"])
        assert e == 0
        assert out.tolist() == c["out"], c


def test_acmove_unit_cases(unit):
    # tests/test_ac_env.py:495-538 (all 12 moves, both flags) and the unit cases' letters 3..6
    for c in unit["acmove"]:
        out, lens, e = O.move(np.array(c["p"]), c["L"], c["move"], c["cyclical"])
        if c["raises"]:
            assert e == {"AssertionError": 1, "IndexError": 2}[c["raises"]], c
        else:
            assert e == 0 and out.tolist() == c["out"] and list(lens) == c["lengths"], c


@pytest.mark.parametrize("L", [7, 18, 36, 128])
@pytest.mark.parametrize("cyc", [1, 0])
def test_transitions(L, cyc):
    d = _load("transitions.npz")
    k = f"L{L}_c{cyc}_"
    s, a = d[k + "state_in"], d[k + "action"]
    out, lens, err = O.move_batch(s, a, L, cyc)
    assert np.array_equal(err, d[k + "err"].astype(np.uint8))
    ok = err == 0
    assert np.array_equal(out[ok], d[k + "state_out"][ok].astype(np.int32))
    assert np.array_equal(lens[ok], d[k + "lengths"][ok].astype(np.int32))


@pytest.mark.parametrize("L", range(1, 10))
def test_smallL_random(L):
    d = _load("smallL_random.npz")
    s, a, c = d[f"L{L}_state_in"], d[f"L{L}_action"], d[f"L{L}_cyclical"]
    exp_out, exp_len, exp_err = d[f"L{L}_state_out"], d[f"L{L}_lengths"], d[f"L{L}_err"]
    for cyc in (0, 1):
        m = c == cyc
        out, lens, err = O.move_batch(s[m], a[m], L, cyc)
        assert np.array_equal(err, exp_err[m].astype(np.uint8))
        ok = err == 0
        assert np.array_equal(out[ok], exp_out[m][ok].astype(np.int32))
        assert np.array_equal(lens[ok], exp_len[m][ok].astype(np.int32))


def test_expand12_goldens():
    d = _load("expand12.npz")
    for tag, L in (("AK3_L36", 36), ("AK2_L7", 7)):
        ch, lens, err = O.expand12(d[tag + "_parents"], L, cyclical=False)
        assert not err.any()
        assert np.array_equal(ch, d[tag + "_children"].astype(np.int32))
        assert np.array_equal(lens, d[tag + "_lengths"].astype(np.int32))


def test_kat_paths():
    with open(os.path.join(GOLDEN, "kat_paths.json")) as f:
        paths = json.load(f)
    for p in paths:
        s = np.array(p["start"], np.int32)
        totals = []
        for a in p["actions"]:
            s, lens, e = O.move(s, p["L"], a, p["cyclical"])
            assert e == 0
            totals.append(sum(lens))
        assert totals == p["totals"], p["name"]
        assert s.tolist() == p["final"]
        assert O.is_trivial(s) == p["trivial"]


def test_env_episodes():
    d = _load("env_episodes.npz")
    L, H = int(d["L"]), int(d["horizon"])
    init = d["initial"].astype(np.int32)
    state = init.copy()
    cnt = np.zeros(init.shape[0], np.int32)
    for t in range(d["actions"].shape[0]):
        r, dn, tr, err, lens, fin = O.env_step(state, d["actions"][t], L, H, cnt, reset_state=init, want_final=True)
        assert not err.any()
        assert np.array_equal(r, d["reward"][t])
        assert np.array_equal(dn, d["done"][t].astype(np.uint8))
        assert np.array_equal(tr, d["truncated"][t].astype(np.uint8))
        assert np.array_equal(fin, d["final_obs"][t].astype(np.int32))
        assert np.array_equal(state, d["obs"][t].astype(np.int32))


def test_config1():
    with open(os.path.join(GOLDEN, "config1.json")) as f:
        rows = json.load(f)
    for row in rows:
        st = np.array([[1, 0, 2, 0]], np.int32)
        cnt = np.zeros(1, np.int32)
        r, dn, tr, err, lens, _ = O.env_step(st, [row["action"]], 2, 1000, cnt)
        assert st[0].tolist() == row["state"]
        assert int(r[0]) == row["reward"] and bool(dn[0]) == row["done"] and bool(tr[0]) == row["truncated"]
        assert lens[0].tolist() == row["lengths"]


def test_features_oracle_vs_reference_golden():
    """oracle/features.py restatement vs the reference's compute_features outputs."""
    from oracle import features as F
    d = np.load(os.path.join(GOLDEN, "features.npz"))
    for L in (18, 36, 7):
        st, exp = d[f"L{L}_states"], d[f"L{L}_features"]
        got = F.compute_features_batch(st, L)
        assert got.dtype == np.float32 and np.array_equal(got.view(np.uint32), exp.view(np.uint32)), L
    tok = F.token_ids(d["L18_states"], 72)
    assert tok.dtype == np.int64 and (tok[:, 36:] == 2).all() and np.array_equal(tok[:, :36], d["L18_states"] + 2)
