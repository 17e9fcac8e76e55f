"""acx.ops.StepPlan (the per-call step with its arguments resolved once) against ops.step on the
same inputs: identical states, counts, rewards, flags, lengths and errors, in place and out of
place, and the lengths-carrying form; argument errors raise at construction or call."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


def _ms_states(L, n):
    import acx
    ms = np.load(os.path.join(os.path.dirname(acx.__file__), "data", "all_presentations.npy"))
    out = np.zeros((n, 2 * L), np.int32)
    for i in range(n):
        p = ms[i % len(ms)]
        out[i, :18], out[i, L: L + 18] = p[:18], p[18:]
    return out


def _bufs(B, L, starts):
    return dict(state=starts.clone(), cnt=torch.zeros(B, dtype=torch.int32, device=DEV),
                rew=torch.zeros(B, dtype=torch.int32, device=DEV), dn=torch.zeros(B, dtype=torch.uint8, device=DEV),
                tr=torch.zeros(B, dtype=torch.uint8, device=DEV), lens=torch.zeros((B, 2), dtype=torch.int32, device=DEV),
                err=torch.zeros(B, dtype=torch.uint8, device=DEV), ec=torch.zeros(1, dtype=torch.int32, device=DEV))


@pytest.mark.parametrize("L,B,lengths_in", [(36, 65536, False), (36, 3000, False), (128, 1000, True), (18, 257, False)])
def test_step_plan_equals_ops_step(L, B, lengths_in):
    from acx import ops
    rows = _ms_states(L, B)
    starts = torch.as_tensor(rows).to(DEV)
    a, b = _bufs(B, L, starts), _bufs(B, L, starts)
    if lengths_in:  # the rows' relator lengths, as VecACEnv keeps them
        lens = np.stack([(rows[:, :L] != 0).sum(1), (rows[:, L:] != 0).sum(1)], 1).astype(np.int32)
        for d in (a, b):
            d["lens"].copy_(torch.as_tensor(lens).to(DEV))
    plan = ops.StepPlan(b["state"], state_out=b["state"], reset_state=starts, step_count=b["cnt"], horizon=7,
                        cyclical=True, reward=b["rew"], done=b["dn"], truncated=b["tr"], lengths=b["lens"],
                        err=b["err"], err_count=b["ec"], lengths_in=lengths_in)
    g = torch.Generator(device=DEV)
    g.manual_seed(L + B)
    for t in range(25):
        act = torch.randint(0, 12, (B,), dtype=torch.int32, device=DEV, generator=g)
        if t == 3:
            act[::97] = 12  # invalid move ids: ACX_ERR_ACTION, state kept
        ops.step(a["state"], act, state_out=a["state"], reset_state=starts, step_count=a["cnt"], horizon=7,
                 cyclical=True, reward=a["rew"], done=a["dn"], truncated=a["tr"], lengths=a["lens"], err=a["err"],
                 err_count=a["ec"], lengths_in=lengths_in)
        assert plan(act) is b["state"]
        for k in a:
            assert torch.equal(a[k], b[k]), (t, k)
    assert int(a["ec"].item()) > 0


def test_step_plan_argument_errors():
    from acx import ops
    L, B = 36, 128
    starts = torch.as_tensor(_ms_states(L, B)).to(DEV)
    st = starts.clone()
    with pytest.raises(ValueError):
        ops.StepPlan(st, step_count=torch.zeros(B + 1, dtype=torch.int32, device=DEV))
    plan = ops.StepPlan(st, reset_state=starts, step_count=torch.zeros(B, dtype=torch.int32, device=DEV), horizon=5)
    with pytest.raises(ValueError):
        plan(torch.zeros(B, dtype=torch.int64, device=DEV))
    with pytest.raises(ValueError):
        plan(torch.zeros(B + 1, dtype=torch.int32, device=DEV))
    with pytest.raises(ValueError):
        ops.StepPlan(st, state_out=starts.clone(), lengths=torch.zeros((B, 2), dtype=torch.int32, device=DEV),
                     lengths_in=True)


def test_stream_handle_is_the_current_stream():
    """ops._stream (the raw current-stream getter every launch uses) names the stream torch
    considers current on the device -- the default one and one entered with torch.cuda.stream --
    and a StepPlan call inside a side stream runs there (its result is ready once that stream is
    synchronised, whatever the default stream does)."""
    from acx import ops
    assert ops._stream(DEV) == torch.cuda.current_stream(DEV).cuda_stream
    assert ops._stream(torch.device("cuda")) == torch.cuda.current_stream().cuda_stream
    side = torch.cuda.Stream(device=DEV)
    with torch.cuda.stream(side):
        assert ops._stream(DEV) == side.cuda_stream
    assert ops._stream(DEV) == torch.cuda.current_stream(DEV).cuda_stream
    L, B = 36, 4096
    starts = torch.as_tensor(_ms_states(L, B)).to(DEV)
    a = _bufs(B, L, starts)
    b = _bufs(B, L, starts)
    act = torch.randint(0, 12, (B,), dtype=torch.int32, device=DEV)
    torch.cuda.synchronize()
    pa = ops.StepPlan(a["state"], reset_state=starts, step_count=a["cnt"], horizon=200, reward=a["rew"])
    pb = ops.StepPlan(b["state"], reset_state=starts, step_count=b["cnt"], horizon=200, reward=b["rew"])
    side.wait_stream(torch.cuda.current_stream(DEV))
    with torch.cuda.stream(side):
        for _ in range(5):
            pa(act)
    for _ in range(5):
        pb(act)
    side.synchronize()
    torch.cuda.synchronize()
    assert torch.equal(a["state"], b["state"]) and torch.equal(a["rew"], b["rew"])
