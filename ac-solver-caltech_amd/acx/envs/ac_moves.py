"""ACMove with the reference's signature (ac_solver/envs/ac_moves.py:159-231), on the GPU.

Move table (ac_moves.py:167-179):
    0: r_1 -> r_1 r_0          1: r_0 -> r_0 r_1^-1      2: r_1 -> r_1 r_0^-1     3: r_0 -> r_0 r_1
    4: r_1 -> x^-1 r_1 x       5: r_0 -> y^-1 r_0 y      6: r_1 -> y^-1 r_1 y     7: r_0 -> x r_0 x^-1
    8: r_1 -> x r_1 x^-1       9: r_0 -> y r_0 y^-1     10: r_1 -> y r_1 y^-1    11: r_0 -> x^-1 r_0 x
Each call is one acx_step launch with B = 1 (plus the host<->device copies); batched
callers use acx.ops.step / acx.ops.expand12 directly.
"""

from __future__ import annotations

import numpy as np
import torch

from .. import _lib, ops


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
    raise ValueError(f"{where}: input outside the acx domain (letters in {{-2..2}}, zeros only as right padding)")


def ACMove(move_id, presentation, max_relator_length, lengths=None, cyclical=True, device=None):
    """Apply AC move `move_id` and reduce; returns (presentation, [n0, n1]).

    `lengths` is accepted for signature compatibility and ignored: the kernel derives the
    lengths from the words (the reference recomputes them too, utils.py:268-281)."""
    assert move_id in range(0, 12), f"Expect n to be in range 0-11 (both inclusive); got {move_id}"
    p = np.asarray(presentation)
    L = int(max_relator_length)
    assert p.shape == (2 * L,), f"presentation must have length 2*max_relator_length = {2 * L}"
    dev = torch.device(device if device is not None else "cuda")
    s = torch.as_tensor(p.astype(np.int32)).reshape(1, 2 * L).to(dev)
    a = torch.tensor([int(move_id)], dtype=torch.int32, device=dev)
    lens = torch.empty((1, 2), dtype=torch.int32, device=dev)
    err = torch.empty((1,), dtype=torch.uint8, device=dev)
    out = ops.step(s, a, cyclical=bool(cyclical), lengths=lens, err=err)
    host = torch.cat([out.reshape(-1), lens.reshape(-1), err.to(torch.int32)]).cpu().numpy()
    raise_for_err(int(host[-1]))
    return host[: 2 * L].astype(p.dtype if p.dtype != np.bool_ else np.int64), [int(host[2 * L]), int(host[2 * L + 1])]
