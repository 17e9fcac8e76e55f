"""CPU restatement of the value-search scoring inputs (TEST INFRASTRUCTURE ONLY: imported by
tests/ as the checker, never by the acx package).

compute_features  restates value_search/feature_extraction.py:11-91 (14 features per
                  presentation: lengths, per-relator letter counts, x exponent sum, length
                  ratio, max/min ratio; ratios as Python float division then float32).
normalise         (f - mean) / std in float32, value_guided_search.py:58-59.
token_ids         value_guided_search.py:68-84: letter + 2 as int64, padded with 2.
Pinned by tests/test_oracle.py against tests/golden/features.npz (made by running the
reference's own compute_features, tests/golden/make_golden.py --features)."""

from __future__ import annotations

import numpy as np


def compute_features(p, L):
    p = np.asarray(p, dtype=np.int8)
    out = np.zeros(14, np.float32)
    n, counts = [], []
    for h in range(2):
        half = p[h * L : (h + 1) * L]
        k = int(np.count_nonzero(half))  # feature_extraction.py:50-51
        w = half[:k]  # :55-56 (the first k entries)
        n.append(k)
        counts.append([int(np.sum(w == v)) for v in (1, -1, 2, -2)])
    tot = n[0] + n[1]
    ex = (counts[0][0] - counts[0][1]) + (counts[1][0] - counts[1][1])
    ratio = n[0] / tot if tot > 0 else 0.5
    mn, mx = min(n), max(n)
    mmr = mx / mn if mn > 0 else mx
    vals = [tot, n[0], n[1], *counts[0], *counts[1], ex, ratio, mmr]
    out[:] = np.array(vals, dtype=np.float32)
    return out


def compute_features_batch(states, L):
    return np.stack([compute_features(s, L) for s in states]) if len(states) else np.zeros((0, 14), np.float32)


def normalise(f, mean, std):
    return (np.asarray(f, np.float32) - np.asarray(mean, np.float32)) / np.asarray(std, np.float32)


def token_ids(states, max_state_dim):
    states = np.asarray(states)
    out = np.full((states.shape[0], max_state_dim), 2, np.int64)
    out[:, : states.shape[1]] = states.astype(np.int64) + 2
    return out
