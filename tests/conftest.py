import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_ROOT = os.path.join(REPO, "ac-solver-caltech_amd")
for p in (REPO, PKG_ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libacx.so on cuda:0)")
    config.addinivalue_line("markers", "slow: longer CPU test")


def unpack_keys_np(keys, L):
    """Packed acx keys (n, kw) uint64 -> (n, 2L) int8 presentations (vectorised, test side)."""
    keys = np.ascontiguousarray(keys, dtype=np.uint64)
    n = keys.shape[0]

    def field(bit, width):
        w, o = bit // 64, bit % 64
        v = keys[:, w] >> np.uint64(o)
        if o + width > 64:
            v = v | (keys[:, w + 1] << np.uint64(64 - o))
        return (v & np.uint64((1 << width) - 1)).astype(np.int64)

    lens = [field(4 * L, 8), field(4 * L + 8, 8)]
    dec = np.array([1, -1, 2, -2], np.int8)
    out = np.zeros((n, 2 * L), np.int8)
    for h in range(2):
        for i in range(L):
            c = field(2 * (h * L + i), 2)
            out[:, h * L + i] = np.where(i < lens[h], dec[c], 0)
    return out


def state_digest(states, checkpoints=()):
    """Rolling sha256 over the int8 bytes of each state in order (tests/golden/make_golden.py
    run_recorded_search): (final digest, {n: digest after n states for n in checkpoints})."""
    import hashlib
    h = hashlib.sha256()
    cps = {}
    want = set(int(c) for c in checkpoints)
    for i, s in enumerate(np.asarray(states, np.int8)):
        h.update(s.tobytes())
        if i + 1 in want:
            cps[str(i + 1)] = h.hexdigest()
    return h.hexdigest(), cps


def in_packed_domain(st, L):
    """rows the packed kernels hold: letters in {-2..2}, zeros only as right padding"""
    ok = ((st >= -2) & (st <= 2)).all(1)
    for h in range(2):
        nz = st[:, h * L:(h + 1) * L] != 0
        n = nz.sum(1)
        ok &= (nz == (np.arange(L)[None, :] < n[:, None])).all(1)
    return ok


def env_step_contract(st, a, cnt, resets, L, H, cyclical=True):
    """One batched env step under acx's error contract (include/acx.h): the oracle's ACMove
    (oracle/acx_oracle.c) for the rows that move; a failed move keeps the state and the step
    count (done = truncated = 0, reward = -(n0+n1)); an out-of-domain row never moves (err 3);
    same-step autoreset to `resets`, an out-of-domain starting row giving err 3.  Mutates st /
    cnt; returns (reward, done, truncated, err)."""
    from oracle import oracle as O
    B = st.shape[0]
    dom = in_packed_domain(st, L)
    out, _, err = O.move_batch(st, a, L, cyclical)
    err = err.copy()
    err[~dom] = 3
    ok = err == 0
    st[ok] = out[ok]
    n = (st[:, :L] != 0).sum(1) + (st[:, L:] != 0).sum(1)
    triv = np.array([ok[b] and O.is_trivial(st[b]) for b in range(B)], dtype=bool)
    cnt[ok] += 1
    trunc = ok & (cnt >= H)
    reward = np.where(triv, H * L * 2, -n).astype(np.int32)
    reset = triv | trunc
    st[reset] = resets[reset]
    cnt[reset] = 0
    err[reset & ~in_packed_domain(st, L)] = 3
    return reward, triv.astype(np.uint8), trunc.astype(np.uint8), err
