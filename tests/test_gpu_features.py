"""GPU parity of the value-search scoring inputs (csrc/acx_features.hip): features and token
ids from int32 presentations and from packed keys, bit-exact against the reference's own
compute_features outputs (tests/golden/features.npz) and the oracle restatement."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import features as F

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


def _bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


@pytest.mark.parametrize("L", [18, 36, 7])
def test_features_states_and_keys_vs_reference(L):
    import acx
    from acx.search._engine import _pack_key
    d = np.load(os.path.join(GOLDEN, "features.npz"))
    st, exp = d[f"L{L}_states"].astype(np.int32), d[f"L{L}_features"]
    f = acx.ops.features(states=torch.as_tensor(st).to(DEV)).cpu().numpy()
    assert np.array_equal(_bits(f), _bits(exp))
    keys = np.stack([_pack_key(s.astype(np.int64), L) for s in st]).view(np.int64)
    fk = acx.ops.features(keys=torch.as_tensor(keys).to(DEV), L=L).cpu().numpy()
    assert np.array_equal(_bits(fk), _bits(exp))
    rng = np.random.default_rng(L)
    mean = rng.normal(size=14).astype(np.float32)
    std = rng.uniform(0.1, 5, size=14).astype(np.float32)
    fn = acx.ops.features(states=torch.as_tensor(st).to(DEV), mean=torch.as_tensor(mean).to(DEV),
                          std=torch.as_tensor(std).to(DEV)).cpu().numpy()
    assert np.array_equal(_bits(fn), _bits(F.normalise(exp, mean, std)))
    for D in (2 * L, 2 * L + 5, 72 if 72 >= 2 * L else 2 * L):
        t = acx.ops.token_ids(states=torch.as_tensor(st).to(DEV), max_state_dim=D).cpu().numpy()
        assert np.array_equal(t, F.token_ids(st, D))
        tk = acx.ops.token_ids(keys=torch.as_tensor(keys).to(DEV), L=L, max_state_dim=D).cpu().numpy()
        assert np.array_equal(tk, F.token_ids(st, D))


@pytest.mark.parametrize("L,cyc", [(36, False), (36, True), (128, False)])
def test_features_of_expand12_keys_equal_features_of_children(L, cyc):
    """The fused scoring path: expand12 packed keys -> features/tokens, without int32 children."""
    import acx
    from oracle import oracle as O
    ms = np.load(os.path.join(os.path.dirname(acx.__file__), "data", "all_presentations.npy"))
    P = np.zeros((700, 2 * L), np.int32)
    for i in range(700):
        p = ms[i % len(ms)]
        P[i, :18], P[i, L : L + 18] = p[:18], p[18:]
    res = acx.ops.expand12(torch.as_tensor(P).to(DEV), cyclical=cyc, keys=True)
    ch, _, err = O.expand12(P, L, cyc)
    ok = err.reshape(-1) == 0
    f = acx.ops.features(keys=res["keys"], L=L).cpu().numpy()[ok]
    exp = F.compute_features_batch(ch.reshape(-1, 2 * L)[ok], L)
    assert np.array_equal(_bits(f), _bits(exp))
    t = acx.ops.token_ids(keys=res["keys"], L=L).cpu().numpy()[ok]
    assert np.array_equal(t, F.token_ids(ch.reshape(-1, 2 * L)[ok], 2 * L))


def test_features_api_edges():
    import acx
    s = torch.zeros((0, 8), dtype=torch.int32, device=DEV)
    assert acx.ops.features(states=s).shape == (0, 14)
    with pytest.raises(ValueError):
        acx.ops.features(states=torch.zeros((2, 8), dtype=torch.int32, device=DEV),
                         keys=torch.zeros((2, 1), dtype=torch.int64, device=DEV), L=4)
    with pytest.raises(ValueError):
        acx.ops.token_ids(states=torch.zeros((2, 8), dtype=torch.int32, device=DEV), max_state_dim=7)
