"""numpy restatement of the reference's per-env ACEnv.step, used as bench.py's CPU baseline.

TEST / BASELINE INFRASTRUCTURE ONLY (never imported by the acx package).

It follows the reference's call structure and numpy call pattern, one env at a time:
ACEnv.step (ac_env.py:91-111) -> ACMove (ac_moves.py:159-231) -> concatenate_relators
(:4-76) / conjugate (:79-156) -> simplify_presentation (utils.py:246-283) ->
simplify_relator (utils.py:178-243) x2 -> is_presentation_trivial (utils.py:57-87):
array copies, non-zero masks, Python while-loops with np.delete, np.pad.  The reference
itself cannot travel to the GPU box, so this restatement stands in for it; bench.py reports
it as cpu_baseline kind "port".  Its speed was calibrated against the reference in the build
container ("CPU baseline").
"""

from __future__ import annotations

import numpy as np


def _valid(p):
    L = len(p) // 2
    ok = len(p) % 2 == 0
    for h in range(2):
        half = p[h * L : (h + 1) * L]
        n = np.count_nonzero(half)
        ok = ok and n > 0 and bool((half[n:] == 0).all())
    return ok


def _reduce_word(word, L, cyclical):
    n = np.count_nonzero(word)
    if len(word) > n:
        assert (word[n:] == 0).all()
    i = 0
    while i < n - 1:
        if word[i] == -word[i + 1]:
            word = np.delete(word, [i, i + 1])
            n -= 2
            i = i - 1 if i else 0
        else:
            i += 1
    if cyclical and n > 0:
        k = 0
        while word[k] == -word[n - k - 1]:
            k += 1
        if k:
            drop = np.concatenate([np.arange(k), n - 1 - np.arange(k)])
            word = np.delete(word, drop)
            n -= 2 * k
    word = np.pad(word, (0, L - len(word)))
    return word, n


def _reduce(p, L, cyclical):
    p = np.array(p)
    assert _valid(p)
    lens = [0, 0]
    for h in range(2):
        w, n = _reduce_word(p[h * L : (h + 1) * L], L, cyclical)
        p[h * L : (h + 1) * L] = w
        lens[h] = n
    return p, lens


def _concat(p, L, i, j, sign):
    p = p.copy()
    a = p[i * L : (i + 1) * L]
    if sign == 1:
        b = p[j * L : (j + 1) * L]
    else:
        b = -p[j * L : (j + 1) * L][::-1]
    a = a[a != 0]
    b = b[b != 0]
    na, nb = len(a), len(b)
    acc = 0
    while acc < min(na, nb) and a[-1 - acc] == -b[acc]:
        acc += 1
    size = na + nb - 2 * acc
    if size <= L:
        p[i * L : i * L + na - acc] = a[: na - acc]
        p[i * L + na - acc : i * L + size] = b[acc:]
        p[i * L + size : (i + 1) * L] = 0
    return p


def _conj(p, L, i, g):
    p = p.copy()
    r = p[i * L : (i + 1) * L]
    r = r[r.nonzero()]
    n = len(r)
    sc = 1 if r[0] == -g else 0
    ec = 1 if r[-1] == g else 0
    size = n + 2 - 2 * (sc + ec)
    if size <= L:
        base = i * L
        p[base + 1 - sc : base + 1 + n - 2 * sc - ec] = r[sc : n - ec]
        if not sc:
            p[base] = g
        if not ec:
            p[base + n + 1 - 2 * sc] = -g
        if sc and ec:
            p[base + size : base + size + 2] = 0
    return p


# move id -> ("cat", i, j, sign) | ("conj", i, g)   (ac_moves.py:167-179)
_MOVES = [("cat", 1, 0, 1), ("cat", 0, 1, -1), ("cat", 1, 0, -1), ("cat", 0, 1, 1),
          ("conj", 1, -1), ("conj", 0, -2), ("conj", 1, -2), ("conj", 0, 1),
          ("conj", 1, 1), ("conj", 0, 2), ("conj", 1, 2), ("conj", 0, -1)]


def ac_move(move_id, p, L, cyclical=True):
    m = _MOVES[move_id]
    p = _concat(p, L, m[1], m[2], m[3]) if m[0] == "cat" else _conj(p, L, m[1], m[2])
    return _reduce(p, L, cyclical)


def _trivial(p):
    if not _valid(p):
        return False
    L = len(p) // 2
    for h in range(2):
        if np.count_nonzero(p[h * L : (h + 1) * L]) != 1:
            return False
    v = np.abs(p[p != 0])
    v.sort()
    return np.array_equal(v, np.arange(1, 3))


class PortEnv:
    """One env: the reference's ACEnv.step semantics with the same per-call numpy work."""

    def __init__(self, initial_state, horizon=1000):
        self.initial = np.array(initial_state)
        self.L = len(self.initial) // 2
        self.horizon = horizon
        self.max_reward = horizon * self.L * 2
        self.reset()

    def reset(self):
        self.state = np.copy(self.initial)
        self.lengths = [int(np.count_nonzero(self.state[h * self.L : (h + 1) * self.L])) for h in range(2)]
        self.count = 0
        self.actions = []
        return self.state

    def step(self, action):
        self.actions += [action]
        self.state, self.lengths = ac_move(action, self.state, self.L)
        done = sum(self.lengths) == 2 and _trivial(self.state)
        reward = self.max_reward * done - sum(self.lengths) * (1 - done)
        self.count += 1
        trunc = self.count >= self.horizon
        return self.state, reward, done, trunc, ({"actions": self.actions.copy()} if done else {})


def run_sample(starts, actions, horizon, seconds):
    """Step len(starts) envs round-robin with the given (T, B) actions, autoresetting on
    done/truncated, until `seconds` elapse.  Returns (env_steps, elapsed_s)."""
    import time

    envs = [PortEnv(s, horizon) for s in starts]
    T, B = actions.shape
    steps = 0
    t0 = time.perf_counter()
    t = 0
    while True:
        for b in range(B):
            _, _, d, tr, _ = envs[b].step(int(actions[t % T, b]))
            if d or tr:
                envs[b].reset()
        steps += B
        t += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            return steps, el
