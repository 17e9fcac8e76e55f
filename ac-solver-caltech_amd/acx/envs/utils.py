"""Presentation helpers with the reference's names and semantics
(ac_solver/envs/utils.py).

Format (utils.py:1-8): a balanced presentation is an even-length array, relator r0 in the
first half and r1 in the second, letters +-1 (x) / +-2 (y), zeros only as right padding.

The setup-time helpers (validation, triviality, padding, conversion) are host numpy; the
word reductions (`simplify_presentation`, `simplify_relator`) run on the GPU through the exact
int32-letter kernels (acx_word_simplify_*, csrc/acx_words.hip), so they accept any integer
letters as the reference does; batched reduction of +-1/+-2 presentations is acx.ops.canonicalize.
"""

from __future__ import annotations

import numpy as np
import torch

from .. import ops


def is_array_valid_presentation(array) -> bool:
    """utils.py:13-54: even length, both relators non-empty, zeros only as right padding."""
    assert isinstance(array, (list, np.ndarray)), f"array must be a list or a numpy array, got {type(array)}"
    a = np.asarray(array)
    if a.ndim != 1 or len(a) % 2 != 0 or len(a) == 0:
        return False
    L = len(a) // 2
    for h in (a[:L], a[L:]):
        n = int(np.count_nonzero(h))
        if n == 0 or np.any(h[n:] != 0):
            return False
    return True


def is_presentation_trivial(presentation) -> bool:
    """utils.py:57-87: valid, both relators of length 1, one x-letter and one y-letter."""
    p = np.asarray(presentation)
    if not is_array_valid_presentation(p):
        return False
    L = len(p) // 2
    if np.count_nonzero(p[:L]) != 1 or np.count_nonzero(p[L:]) != 1:
        return False
    return sorted(int(abs(v)) for v in p[p != 0]) == [1, 2]


def generate_trivial_states(max_relator_length: int) -> np.ndarray:
    """utils.py:91-114: the 8 trivial presentations, shape (8, 2L)."""
    L = int(max_relator_length)
    out = np.zeros((8, 2 * L), dtype=np.int64)
    row = 0
    for g in (1, 2):
        for s1 in (-1, 1):
            for s2 in (-1, 1):
                out[row, 0] = s1 * g
                out[row, L] = s2 * (3 - g)
                row += 1
    return out


def convert_relators_to_presentation(relator1, relator2, max_relator_length) -> np.ndarray:
    """utils.py:117-148: two zero-free relators -> int8 presentation padded to L."""
    assert 0 not in list(relator1) and 0 not in list(relator2), "relator1 and relator2 must not be padded with zeros."
    assert max_relator_length >= max(len(relator1), len(relator2)), (
        "max_relator_length must be greater than or equal to the lengths of relator1 and rel2."
    )
    L = int(max_relator_length)
    out = np.zeros(2 * L, dtype=np.int8)
    out[: len(relator1)] = list(relator1)
    out[L : L + len(relator2)] = list(relator2)
    return out


def change_max_relator_length_of_presentation(presentation, new_max_length) -> np.ndarray:
    """utils.py:151-175: re-pad a presentation to a new max_relator_length (int8)."""
    p = np.asarray(presentation)
    L0 = len(p) // 2
    n0 = int(np.count_nonzero(p[:L0]))
    n1 = int(np.count_nonzero(p[L0:]))
    return convert_relators_to_presentation(p[:n0], p[L0 : L0 + n1], new_max_length)


def _device(device):
    return torch.device(device if device is not None else "cuda")


def simplify_presentation(presentation, max_relator_length, lengths_of_words=None, cyclical=True, device=None):
    """utils.py:246-283 on the GPU (acx_word_simplify_presentation: exact on any integer letters).
    Returns (presentation, [n0, n1]); raises AssertionError for an invalid presentation, as the
    reference does."""
    p = np.array(presentation)
    L = int(max_relator_length)
    assert is_array_valid_presentation(p), (
        f"{p} is not a valid presentation. Expect all zeros to be padded to the right."
    )
    assert len(p) == 2 * L
    t = torch.as_tensor(p.astype(np.int32)).reshape(1, 2 * L).to(_device(device))
    out, lens, err = ops.word_simplify_presentation(t, cyclical=bool(cyclical))
    host = torch.cat([out.reshape(-1), lens.reshape(-1), err.to(torch.int32)]).cpu().numpy()
    _raise(int(host[-1]))
    return host[: 2 * L].astype(p.dtype), [int(host[2 * L]), int(host[2 * L + 1])]


def _raise(code: int) -> None:
    from .ac_moves import raise_for_err
    raise_for_err(code, "simplify")


def simplify_relator(relator, max_relator_length, cyclical=False, padded=True, device=None):
    """utils.py:178-243 on the GPU (acx_word_simplify_relator: exact on any integer letters, and on
    arrays longer than max_relator_length).  Returns (relator, length) like the reference: the
    reduced array, padded with zeros to max_relator_length when `padded`, else the array after the
    deletions (its trailing zeros included)."""
    assert isinstance(relator, np.ndarray), "expect relator to be a numpy array"
    r = relator
    m = int(r.shape[0])
    L = int(max_relator_length)
    t = torch.as_tensor(r.astype(np.int32)).reshape(1, m).to(_device(device))
    out, ol, n, err = ops.word_simplify_relator(t, L, cyclical=bool(cyclical), padded=bool(padded))
    w = out.shape[1]
    host = torch.cat([out.reshape(-1), ol, n, err.to(torch.int32)]).cpu().numpy()
    _raise(int(host[-1]))
    return host[: int(host[w])].astype(r.dtype), int(host[w + 1])
