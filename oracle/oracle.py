"""ctypes wrapper around liboracle.so (oracle/acx_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, as the checker.  The product (the ``acx`` package / libacx.so) never
imports this module.
"""

from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
# tests/test_sanitizers.py runs the oracle's own tests against the ASan + UBSan build
# (liboracle_asan.so) by naming it here
LIB_PATH = os.environ.get("ACX_ORACLE_LIB", LIB_PATH)

ERR_OK, ERR_INVALID, ERR_EMPTY_CONJ, ERR_DOMAIN, ERR_BAD_ACTION, ERR_OTHER = 0, 1, 2, 3, 4, 9

_lib = None


def build(force: bool = False) -> str:
    if os.path.basename(LIB_PATH) != "liboracle.so":
        return LIB_PATH  # a sanitizer build, made by its caller
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(
        os.path.join(HERE, "acx_oracle.c")
    ):
        subprocess.check_call(["make", "-s", "-C", HERE, "liboracle.so"])
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB_PATH)
        i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
        u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
        c = ctypes
        L.acx_oracle_move.argtypes = [i32p, c.c_int32, c.c_int32, c.c_int32, i32p, i32p]
        L.acx_oracle_move.restype = c.c_int
        L.acx_oracle_move_batch.argtypes = [i32p, i32p, c.c_int64, c.c_int32, c.c_int32, i32p, i32p, u8p]
        L.acx_oracle_move_batch.restype = None
        L.acx_oracle_expand12.argtypes = [i32p, c.c_int64, c.c_int32, c.c_int32, i32p, i32p, u8p]
        L.acx_oracle_expand12.restype = None
        L.acx_oracle_simplify_relator.argtypes = [i32p, c.c_int32, c.c_int32, c.c_int32, c.c_int32, i32p,
                                                  c.POINTER(c.c_int32), c.POINTER(c.c_int32)]
        L.acx_oracle_simplify_relator.restype = c.c_int
        L.acx_oracle_simplify_presentation.argtypes = [i32p, c.c_int32, c.c_int32, i32p]
        L.acx_oracle_simplify_presentation.restype = c.c_int
        L.acx_oracle_concatenate.argtypes = [i32p, c.c_int32, c.c_int32, c.c_int32, c.c_int32]
        L.acx_oracle_concatenate.restype = c.c_int
        L.acx_oracle_conjugate.argtypes = [i32p, c.c_int32, c.c_int32, c.c_int32, c.c_int32]
        L.acx_oracle_conjugate.restype = c.c_int
        L.acx_oracle_is_valid.argtypes = [i32p, c.c_int32]
        L.acx_oracle_is_valid.restype = c.c_int
        L.acx_oracle_is_trivial.argtypes = [i32p, c.c_int32]
        L.acx_oracle_is_trivial.restype = c.c_int
        L.acx_oracle_env_step.argtypes = [i32p, i32p, c.c_int64, c.c_int32, c.c_int32, c.c_int32,
                                          c.c_void_p, i32p, i32p, u8p, u8p, c.c_void_p, c.c_void_p, u8p]
        L.acx_oracle_env_step.restype = None
        _lib = L
    return _lib


def _i32(a):
    return np.ascontiguousarray(np.asarray(a), dtype=np.int32)


def move(state, L, action, cyclical=True):
    """ACMove restated: returns (out_state int32 (2L,), [n0, n1], err)."""
    s = _i32(state).copy()
    out = np.empty_like(s)
    lens = np.zeros(2, np.int32)
    e = lib().acx_oracle_move(s, int(L), int(action), int(cyclical), out, lens)
    return out, [int(lens[0]), int(lens[1])], int(e)


def move_batch(states, actions, L, cyclical=True):
    s = _i32(states).reshape(-1, 2 * L)
    a = _i32(actions).reshape(-1)
    B = s.shape[0]
    out = np.empty_like(s)
    lens = np.zeros((B, 2), np.int32)
    err = np.zeros(B, np.uint8)
    lib().acx_oracle_move_batch(s, a, B, int(L), int(cyclical), out, lens, err)
    return out, lens, err


def expand12(parents, L, cyclical=False):
    p = _i32(parents).reshape(-1, 2 * L)
    N = p.shape[0]
    ch = np.empty((N, 12, 2 * L), np.int32)
    lens = np.zeros((N, 12, 2), np.int32)
    err = np.zeros((N, 12), np.uint8)
    lib().acx_oracle_expand12(p, N, int(L), int(cyclical), ch, lens, err)
    return ch, lens, err


def simplify_relator(relator, L, cyclical=False, padded=True):
    r = _i32(relator)
    m = r.shape[0]
    out = np.zeros(max(m, L, 1), np.int32)
    ol, n = ctypes.c_int32(0), ctypes.c_int32(0)
    e = lib().acx_oracle_simplify_relator(r, m, int(L), int(cyclical), int(padded), out,
                                          ctypes.byref(ol), ctypes.byref(n))
    return out[: ol.value], int(n.value), int(e)


def simplify_presentation(p, L, cyclical=True):
    s = _i32(p).copy()
    lens = np.zeros(2, np.int32)
    e = lib().acx_oracle_simplify_presentation(s, int(L), int(cyclical), lens)
    return s, [int(lens[0]), int(lens[1])], int(e)


def concatenate(p, L, i, j, sign):
    s = _i32(p).copy()
    lib().acx_oracle_concatenate(s, int(L), int(i), int(j), int(sign))
    return s


def conjugate(p, L, i, j, sign):
    s = _i32(p).copy()
    e = lib().acx_oracle_conjugate(s, int(L), int(i), int(j), int(sign))
    return s, int(e)


def is_valid(p):
    s = _i32(p)
    if s.size == 0:
        return False
    return bool(lib().acx_oracle_is_valid(s, s.shape[0]))


def is_trivial(p):
    s = _i32(p)
    if s.size == 0:
        return False
    return bool(lib().acx_oracle_is_trivial(s, s.shape[0]))


def env_step(state, actions, L, horizon, step_count, reset_state=None, cyclical=True, want_final=False):
    """Batched ACEnv.step with same-step autoreset; mutates state and step_count in place."""
    B = state.shape[0]
    assert state.dtype == np.int32 and state.flags.c_contiguous
    assert step_count.dtype == np.int32
    a = _i32(actions)
    reward = np.zeros(B, np.int32)
    done = np.zeros(B, np.uint8)
    trunc = np.zeros(B, np.uint8)
    err = np.zeros(B, np.uint8)
    lens = np.zeros((B, 2), np.int32)
    final = np.zeros_like(state) if want_final else None
    rs = None
    if reset_state is not None:
        reset_state = _i32(reset_state)
        rs = reset_state.ctypes.data
    lib().acx_oracle_env_step(state, a, B, int(L), int(horizon), int(cyclical), rs, step_count, reward, done,
                              trunc, final.ctypes.data if final is not None else None, lens.ctypes.data, err)
    return reward, done, trunc, err, lens, final
