"""ac_solver/envs/ac_moves.py's functions with the reference's signatures, on the GPU.

Move table (ac_moves.py:167-179):
    0: r_1 -> r_1 r_0          1: r_0 -> r_0 r_1^-1      2: r_1 -> r_1 r_0^-1     3: r_0 -> r_0 r_1
    4: r_1 -> x^-1 r_1 x       5: r_0 -> y^-1 r_0 y      6: r_1 -> y^-1 r_1 y     7: r_0 -> x r_0 x^-1
    8: r_1 -> x r_1 x^-1       9: r_0 -> y r_0 y^-1     10: r_1 -> y r_1 y^-1    11: r_0 -> x^-1 r_0 x

ACMove on a presentation of letters +-1 / +-2 with zeros only as right padding is one acx_step
launch (the packed 2-bit kernels); any other input -- letters beyond +-2 (the reference's word
functions are generator-agnostic, its unit tests use 3..6) or zeros inside a relator -- goes to
acx_word_move, the exact int32-letter kernel.  concatenate_relators / conjugate (the moves
without the reduction) are acx_concatenate / acx_conjugate.  Each call is one B = 1 launch plus
the host<->device copies; batched callers use acx.ops directly.
"""

from __future__ import annotations

import threading

import numpy as np
import torch

from .. import _lib, ops

# Per-thread staging for the per-call ACMove (B = 1): one pinned host block in, one device block
# holding the kernel's outputs (state | lengths | error byte), one pinned host block out -- so a
# call is one H2D copy, one step launch and one D2H copy, with no allocations and no extra
# conversion kernels.  Thread-local: ACMove is re-entrant in the reference.
_TLS = threading.local()


def _stage(dev: torch.device, L: int):
    cache = getattr(_TLS, "stage", None)
    if cache is None:
        cache = _TLS.stage = {}
    key = (dev.type, dev.index if dev.index is not None else torch.cuda.current_device(), L)
    st = cache.get(key)
    if st is None:
        n = 2 * L + 3  # state 2L, lengths 2, error byte (in an int32 slot)
        h_in = torch.empty(2 * L + 1, dtype=torch.int32, pin_memory=True)
        d_in = torch.empty(2 * L + 1, dtype=torch.int32, device=dev)
        d_out = torch.zeros(n, dtype=torch.int32, device=dev)
        h_out = torch.empty(n, dtype=torch.int32, pin_memory=True)
        st = cache[key] = (h_in, d_in, d_out, h_out)
    return st


def raise_for_err(code: int, where: str = "ACMove") -> None:
    """Map an acx per-env error code to the exception the reference raises."""
    if code == _lib.ERR_NONE:
        return
    if code == _lib.ERR_INVALID:
        raise AssertionError(f"{where}: presentation is not valid after the move (utils.py:264-266)")
    if code == _lib.ERR_EMPTY_CONJ:
        raise IndexError(f"{where}: conjugating an empty relator (ac_moves.py:119)")
    if code == _lib.ERR_ACTION:
        raise AssertionError(f"{where}: move id must be in range 0-11 (ac_moves.py:188)")
    if code == _lib.ERR_PAD:
        raise ValueError(f"{where}: relator longer than max_relator_length (np.pad, utils.py:235-236)")
    raise ValueError(f"{where}: input outside the acx domain (letters in {{-2..2}}, zeros only as right padding)")


def in_packed_domain(p: np.ndarray, L: int) -> bool:
    """Letters in {-2..2} with zeros only as right padding: the packed kernels' domain."""
    if p.shape != (2 * L,) or np.any(np.abs(p) > 2):
        return False
    for h in range(2):
        r = p[h * L : (h + 1) * L]
        n = int(np.count_nonzero(r))
        if np.any(r[n:] != 0):
            return False
    return True


def _device(device):
    return torch.device(device if device is not None else "cuda")


def _out_dtype(p: np.ndarray):
    return p.dtype if p.dtype != np.bool_ else np.int64


def ACMove(move_id, presentation, max_relator_length, lengths=None, cyclical=True, device=None):
    """Apply AC move `move_id` and reduce; returns (presentation, [n0, n1]).

    `lengths` is accepted for signature compatibility and not read: the reference recomputes the
    lengths from the words too (utils.py:268-281)."""
    assert move_id in range(0, 12), f"Expect n to be in range 0-11 (both inclusive); got {move_id}"
    p = np.asarray(presentation)
    L = int(max_relator_length)
    assert p.shape == (2 * L,), f"presentation must have length 2*max_relator_length = {2 * L}"
    dev = _device(device)
    if in_packed_domain(p, L):
        h_in, d_in, d_out, h_out = _stage(dev, L)
        hv = h_in.numpy()
        hv[: 2 * L] = p
        hv[2 * L] = int(move_id)
        d_in.copy_(h_in, non_blocking=True)
        # the kernel always writes the error byte; the slot's other bytes stay 0 from allocation
        err = d_out.view(torch.uint8)[4 * (2 * L + 2) : 4 * (2 * L + 2) + 1]
        ops.step(d_in[: 2 * L].view(1, 2 * L), d_in[2 * L :], state_out=d_out[: 2 * L].view(1, 2 * L),
                 cyclical=bool(cyclical), lengths=d_out[2 * L : 2 * L + 2].view(1, 2), err=err)
        h_out.copy_(d_out, non_blocking=True)
        torch.cuda.current_stream(dev).synchronize()
        host = h_out.numpy()
        # the error byte is the low byte of the last int32 slot (little-endian)
        raise_for_err(int(host[2 * L + 2]) & 0xff)
        return host[: 2 * L].astype(_out_dtype(p)), [int(host[2 * L]), int(host[2 * L + 1])]
    s = torch.as_tensor(p.astype(np.int32)).reshape(1, 2 * L).to(dev)
    a = torch.tensor([int(move_id)], dtype=torch.int32, device=dev)
    out, lens, _, err = ops.word_move(s, a, cyclical=bool(cyclical))
    host = torch.cat([out.reshape(-1), lens.reshape(-1), err.to(torch.int32)]).cpu().numpy()
    raise_for_err(int(host[-1]))
    return host[: 2 * L].astype(_out_dtype(p)), [int(host[2 * L]), int(host[2 * L + 1])]


def _pair(p, L, lengths, device):
    dev = _device(device)
    s = torch.as_tensor(p.astype(np.int32)).reshape(1, 2 * L).to(dev)
    ln = torch.tensor([[int(lengths[0]), int(lengths[1])]], dtype=torch.int32, device=dev)
    return s, ln, dev


def concatenate_relators(presentation, max_relator_length, i, j, sign, lengths, device=None):
    """ac_moves.py:4-76 (acx_concatenate): r_i <- r_i r_j^{sign}, junction cancellation only.
    Returns (presentation, lengths); like the reference, a move that fits writes lengths[i] of
    the list it was given (:65)."""
    assert all([i in [0, 1], j in [0, 1], i == 1 - j]), (
        f"expect i and j to be 0 or 1 and i != j; got i = {i}, j = {j}")
    assert sign in [1, -1], f"expect sign to be +1 or -1, received {sign}"
    p = np.asarray(presentation)
    L = int(max_relator_length)
    assert p.shape == (2 * L,), f"presentation must have length 2*max_relator_length = {2 * L}"
    s, ln, dev = _pair(p, L, lengths, device)
    out, lo = ops.concatenate(s, i, j, sign, lengths=ln)
    host = torch.cat([out.reshape(-1), lo.reshape(-1)]).cpu().numpy()
    new_i = int(host[2 * L + i])  # the new size when the move fits, else the given value
    if new_i != int(lengths[i]):
        lengths[i] = new_i
    return host[: 2 * L].astype(_out_dtype(p)), lengths


def conjugate(presentation, max_relator_length, i, j, sign, lengths, device=None):
    """ac_moves.py:79-156 (acx_conjugate): r_i <- x_j^{sign} r_i x_j^{-sign}, end cancellation
    only.  Returns (presentation, lengths): the given lengths with [i] replaced by the new size
    when the move fits (the reference returns a copy then, :127)."""
    assert all([i in [0, 1], j in [1, 2]]), f"expect i to be 0 and 1 and j to be 1 or 2; got i = {i}, j = {j}"
    assert sign in [1, -1], f"expect sign to be +1 or -1, received {sign}"
    p = np.asarray(presentation)
    L = int(max_relator_length)
    assert p.shape == (2 * L,), f"presentation must have length 2*max_relator_length = {2 * L}"
    s, ln, dev = _pair(p, L, lengths, device)
    out, lo, err = ops.conjugate(s, i, j, sign, lengths=ln)
    host = torch.cat([out.reshape(-1), lo.reshape(-1), err.to(torch.int32)]).cpu().numpy()
    raise_for_err(int(host[-1]), "conjugate")
    return host[: 2 * L].astype(_out_dtype(p)), [int(host[2 * L]), int(host[2 * L + 1])]
