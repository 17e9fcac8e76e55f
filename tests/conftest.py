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
