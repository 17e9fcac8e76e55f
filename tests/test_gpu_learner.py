"""GPU parity of the PPO rollout plumbing (acx_step_learner + acx_curriculum_assign, via
acx.agents.LearnerEnv) against oracle/curriculum.py, the restatement of the env side of
training.py:221-352 (oracle env step, episode action lists, round-1 curriculum)."""
import os

import numpy as np
import pytest
import torch

from oracle import curriculum as C

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


def _ms_states(L, n):
    import acx
    ms = np.load(os.path.join(os.path.dirname(acx.__file__), "data", "all_presentations.npy"))
    out = np.zeros((n, 2 * L), np.int32)
    for i in range(n):
        p = ms[i % len(ms)]
        out[i, :18], out[i, L : L + 18] = p[:18], p[18:]
    return out


@pytest.mark.parametrize("L,B,N,H,T,adtype", [(36, 128, 300, 5, 40, torch.int64), (36, 1000, 1190, 9, 30, torch.int32),
                                              (18, 77, 200, 3, 60, torch.int64), (128, 64, 150, 4, 25, torch.int64)])
def test_learner_env_matches_training_loop_restatement(L, B, N, H, T, adtype):
    from acx.agents import LearnerEnv
    init = _ms_states(L, N)
    # a few envs that solve quickly: trivial-adjacent starts ([x],[y x]) so `done` happens too
    init[1] = 0
    init[1, 0], init[1, L], init[1, L + 1] = 1, 2, 1
    ref = C.RolloutEnvs(init, B, H)
    env = LearnerEnv(init, B, horizon_length=H, device=DEV)
    obs = torch.empty((T + 1, B, 2 * L), dtype=torch.float32, device=DEV)
    rew = torch.empty((T, B), dtype=torch.float32, device=DEV)
    dones = torch.empty((T, B), dtype=torch.float32, device=DEV)
    env.initial_obs(out=obs[0])
    rng = np.random.default_rng(L + B)
    host_pick = lambda i: (7 * i + 3) % N  # noqa: E731  stands in for random.choice (training.py:337-346)
    n_host = n_done = 0
    for t in range(T):
        a = rng.integers(0, 12, size=B)
        res = ref.step(a, host_pick)
        done, trunc, ep_len, needs_host = env.step(torch.as_tensor(a).to(DEV, adtype), obs_out=obs[t + 1],
                                                   reward_out=rew[t], done_out=dones[t])
        nh = needs_host.cpu().numpy().astype(bool)
        assert np.array_equal(nh, res["picked_by_host"]), t
        for i in np.nonzero(nh)[0]:
            env.place(int(i), host_pick(int(i)), obs_out=obs[t + 1])
        n_host += int(nh.sum())
        assert np.array_equal(done.cpu().numpy(), res["done"]) and np.array_equal(trunc.cpu().numpy(), res["truncated"])
        assert np.array_equal(rew[t].cpu().numpy(), res["reward"].astype(np.float32))
        assert np.array_equal(dones[t].cpu().numpy(), res["done"].astype(np.float32))
        assert np.array_equal(ep_len.cpu().numpy(), res["episode_len"])
        many = env.episode_actions_many(list(res["info_actions"].keys()))
        for i, acts in res["info_actions"].items():
            assert env.episode_actions(i) == acts and many[i] == acts
            n_done += 1
        assert np.array_equal(env.state.cpu().numpy(), ref.state), t
        assert np.array_equal(obs[t + 1].cpu().numpy(), ref.state.astype(np.float32)), t
        assert env.curr_index.cpu().tolist() == ref.curr_states
    assert n_host > 0 or N - B > T * B  # round 1 completed in the long cases


@pytest.mark.parametrize("L,B,N,H", [(36, 5000, 9000, 6), (36, 4096, 4200, 3), (128, 300, 700, 4), (18, 65, 90, 2),
                                     (19, 333, 700, 3)])  # odd L: the curriculum copy's per-int32 path
def test_fused_learner_step_equals_two_calls(L, B, N, H):
    """acx_learner_step (step kernel + one curriculum pass from per-wave counts) gives the same
    state, outputs, curriculum indices and host flags as acx_step_learner + acx_curriculum_assign,
    across round-1 completion (full tiles, partial last tile and block, several L)."""
    from acx.agents import LearnerEnv
    init = _ms_states(L, N)
    init[3] = 0
    init[3, 0], init[3, L], init[3, L + 1] = 1, 2, 1  # solves in one move: done events
    ea = LearnerEnv(init, B, horizon_length=H, device=DEV)
    eb = LearnerEnv(init, B, horizon_length=H, device=DEV)
    T = 3 * H + 2 * (N - B) // max(1, B // H) + 4
    g = torch.Generator(device=DEV)
    g.manual_seed(L + B)
    outs = [[torch.empty((B, 2 * L), dtype=torch.float32, device=DEV), torch.empty(B, dtype=torch.float32, device=DEV),
             torch.empty(B, dtype=torch.float32, device=DEV)] for _ in range(2)]
    hosted = 0
    for t in range(T):
        a = torch.randint(0, 12, (B,), dtype=torch.int64, device=DEV, generator=g)
        ra = ea.step(a, *outs[0], fused=True)
        rb = eb.step(a, *outs[1], fused=False)
        for x, y in zip(ra, rb):
            assert torch.equal(x, y), t
        for x, y in zip(outs[0], outs[1]):
            assert torch.equal(x, y), t
        assert torch.equal(ea.state, eb.state) and torch.equal(ea.vec.reset_state, eb.vec.reset_state), t
        assert torch.equal(ea.curr_index, eb.curr_index) and torch.equal(ea.next_index, eb.next_index), t
        nh = ra[3].cpu().numpy().nonzero()[0]
        for i in nh[:50]:
            ea.place(int(i), int(i) % N, obs_out=outs[0][0])
            eb.place(int(i), int(i) % N, obs_out=outs[1][0])
        for i in nh[50:]:
            ea.needs_host[int(i)] = 0
            eb.needs_host[int(i)] = 0
        hosted += len(nh)
    assert int(ea.next_index.item()) == N and hosted > 0


def test_step_learner_matches_acx_step():
    """obs_f32 / reward_f32 / done_f32 are the int outputs of acx_step, converted."""
    import acx
    from acx import _lib
    L, B = 36, 5000
    init = _ms_states(L, B)
    st_a = torch.as_tensor(init).to(DEV)
    st_b = st_a.clone()
    rs = st_a.clone()
    ca = torch.zeros(B, dtype=torch.int32, device=DEV)
    cb = ca.clone()
    lib = _lib.load()
    stream = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device=DEV)
    g.manual_seed(1)
    for t in range(30):
        a = torch.randint(0, 12, (B,), dtype=torch.int64, device=DEV, generator=g)
        rew = torch.empty(B, dtype=torch.int32, device=DEV)
        dn = torch.empty(B, dtype=torch.uint8, device=DEV)
        acx.ops.step(st_a, a.to(torch.int32), state_out=st_a, reset_state=rs, step_count=ca, horizon=11, reward=rew,
                     done=dn)
        obs = torch.empty((B, 2 * L), dtype=torch.float32, device=DEV)
        rf = torch.empty(B, dtype=torch.float32, device=DEV)
        df = torch.empty(B, dtype=torch.float32, device=DEV)
        rc = lib.acx_step_learner(st_b.data_ptr(), None, a.data_ptr(), rs.data_ptr(), cb.data_ptr(), obs.data_ptr(),
                                  rf.data_ptr(), df.data_ptr(), None, None, None, 0, None, 0, None, None, None, None, B,
                                  L, 11, 1, stream)
        assert rc == 0
        assert torch.equal(st_a, st_b) and torch.equal(ca, cb)
        assert torch.equal(obs, st_b.to(torch.float32))
        assert torch.equal(rf, rew.to(torch.float32)) and torch.equal(df, dn.to(torch.float32))
    # out-of-range int64 action -> ACX_ERR_ACTION, state kept
    err = torch.zeros(B, dtype=torch.uint8, device=DEV)
    bad = torch.full((B,), 12, dtype=torch.int64, device=DEV)
    before = st_b.clone()
    assert lib.acx_step_learner(st_b.data_ptr(), None, bad.data_ptr(), rs.data_ptr(), cb.data_ptr(), None, None, None,
                                None, None, None, 0, None, 0, None, None, err.data_ptr(), None, B, L, 11, 1,
                                stream) == 0
    assert (err == _lib.ERR_ACTION).all() and torch.equal(before, st_b)


def _curriculum_cases():
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_curriculum_golden import golden_cases
    return golden_cases()


@pytest.mark.parametrize("case", _curriculum_cases(), ids=lambda c: c[0])
@pytest.mark.parametrize("fused", [True, False])
def test_learner_env_matches_reference_training_loop(case, fused):
    """LearnerEnv + CurriculumRecord against the reference's own ppo_training_loop run
    (tests/golden/curriculum.npz): every step's rewards / done / truncated, the float32 next_obs
    row buffer (post autoreset and curriculum restart), curr_states, and the final
    success_record / ACMoves_hist / states_processed -- round-2 draws from `random` seeded as
    the trainer seeds it (training.py:204)."""
    import random

    from acx.agents import CurriculumRecord, LearnerEnv
    from test_curriculum_golden import check_final
    name, m, g = case
    init = g["initial_states"].astype(np.int32)
    B, T, U, L = m["num_envs"], m["num_steps"], m["updates"], init.shape[1] // 2
    env = LearnerEnv(init, B, horizon_length=m["horizon"], device=DEV)
    rng = random.Random()
    rec = CurriculumRecord(len(init), B, m["repeat_solved_prob"], rng=rng)
    obs = torch.empty((B, 2 * L), dtype=torch.float32, device=DEV)
    rew = torch.empty(B, dtype=torch.float32, device=DEV)
    nd = torch.empty(B, dtype=torch.float32, device=DEV)
    for u in range(1, U + 1):
        rng.seed(m["seed"] + u)
        for s in range(T):
            t = (u - 1) * T + s
            a = torch.as_tensor(g["actions"][t].astype(np.int64)).to(DEV)
            done, trunc, _, needs_host = env.step(a, obs_out=obs, reward_out=rew, done_out=nd, fused=fused)
            rec.process(env, done, trunc, needs_host, obs_out=obs)
            assert np.array_equal(rew.cpu().numpy(), g["reward"][t].astype(np.float32)), (name, t)
            assert np.array_equal(done.cpu().numpy(), g["done"][t]) and np.array_equal(trunc.cpu().numpy(),
                                                                                     g["truncated"][t]), (name, t)
            assert rec.curr_states == list(g["curr_states"][t]), (name, t)
            assert env.curr_index.cpu().tolist() == rec.curr_states, (name, t)
            assert np.array_equal(obs.cpu().numpy(), g["post_state"][t].astype(np.float32)), (name, t)
            assert np.array_equal(env.state.cpu().numpy(), g["post_state"][t].astype(np.int32)), (name, t)
    check_final(rec, m)


def test_fused_learner_step_full_size_lookback():
    """The fused step's look-back at a full per-GPU batch (2^20 envs = 16,384 tiles, two resident
    rounds): desynchronised episodes (about B/H finished envs per step, scattered), then a step
    where every env finishes (the whole batch ranked in one launch) across round-1 completion --
    state, outputs, curriculum indices, next_index and host flags equal to the four-launch path
    (acx_step_learner + acx_curriculum_assign)."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import ms_starts
    from acx.agents import LearnerEnv
    L, B, H = 36, 1 << 20, 7
    N = B + (H + 2) * B // H + B // 2  # round 1 completes inside the all-finish step
    init = ms_starts(L, N)
    ea = LearnerEnv(init, B, horizon_length=H, device=DEV)
    eb = LearnerEnv(init, B, horizon_length=H, device=DEV)
    desync = (torch.arange(B, dtype=torch.int32, device=DEV) * 5) % H
    ea.vec.step_count.copy_(desync)
    eb.vec.step_count.copy_(desync)
    g = torch.Generator(device=DEV)
    g.manual_seed(7)
    outs = [[torch.empty((B, 2 * L), dtype=torch.float32, device=DEV), torch.empty(B, dtype=torch.float32, device=DEV),
             torch.empty(B, dtype=torch.float32, device=DEV)] for _ in range(2)]
    n_fin = []
    for t in range(2 * H + 2):
        if t == H + 1:  # every env finishes on this step
            ea.vec.step_count.fill_(H - 1)
            eb.vec.step_count.fill_(H - 1)
        a = torch.randint(0, 12, (B,), dtype=torch.int64, device=DEV, generator=g)
        ra = ea.step(a, *outs[0], fused=True)
        rb = eb.step(a, *outs[1], fused=False)
        for x, y in zip(ra, rb):
            assert torch.equal(x, y), t
        for x, y in zip(outs[0], outs[1]):
            assert torch.equal(x, y), t
        assert torch.equal(ea.state, eb.state) and torch.equal(ea.vec.reset_state, eb.vec.reset_state), t
        assert torch.equal(ea.curr_index, eb.curr_index) and torch.equal(ea.next_index, eb.next_index), t
        n_fin.append(int((ra[0] | ra[1]).sum().item()))
        nh = ra[3] != 0
        ea.needs_host[nh] = 0
        eb.needs_host[nh] = 0
    assert n_fin[H + 1] == B and int(ea.next_index.item()) == N
    assert min(n_fin[: H]) > B // (2 * H)
    del ea, eb, outs
    torch.cuda.empty_cache()


def test_fused_learner_step_out_of_domain_curriculum_row():
    """A curriculum row outside the packed domain is taken as it is by both paths (the fused step's
    tail copies the row, as acx_curriculum_assign does); later steps report it as err 3 on both,
    the state, observation and reset rows staying that row's exact values."""
    from acx.agents import CurriculumRecord, LearnerEnv
    L, B, N, H = 36, 256, 900, 2
    init = _ms_states(L, N)
    for k in (B + 3, B + 70, B + 300):
        init[k, 5] = 3  # a letter outside +-1 / +-2
    init[B + 130, 1] = 0  # a zero inside relator 0
    ea = LearnerEnv(init, B, horizon_length=H, device=DEV)
    eb = LearnerEnv(init, B, horizon_length=H, device=DEV)
    ra_rec = CurriculumRecord(N, B, 0.5)
    rb_rec = CurriculumRecord(N, B, 0.5)
    g = torch.Generator(device=DEV)
    g.manual_seed(3)
    errs = 0
    for t in range(2 * H + 1):
        a = torch.randint(0, 12, (B,), dtype=torch.int64, device=DEV, generator=g)
        oa = torch.empty((B, 2 * L), dtype=torch.float32, device=DEV)
        ob = torch.empty((B, 2 * L), dtype=torch.float32, device=DEV)
        da, ta, _, ha = ea.step(a, obs_out=oa, fused=True)
        db, tb, _, hb = eb.step(a, obs_out=ob, fused=False)
        assert torch.equal(ha, hb), t
        errs += int((ea.vec.err == 3).sum().item())
        assert torch.equal(ea.vec.err, eb.vec.err), t
        pa = ra_rec.process(ea, da, ta, ha, obs_out=oa)
        pb = rb_rec.process(eb, db, tb, hb, obs_out=ob)
        assert pa == pb, t
        assert torch.equal(ea.state, eb.state) and torch.equal(ea.vec.reset_state, eb.vec.reset_state), t
        assert torch.equal(oa, ob) and torch.equal(ea.curr_index, eb.curr_index), t
        assert torch.equal(ea.vec.step_count, eb.vec.step_count), t
    assert errs > 0  # the copied out-of-domain rows were stepped (err 3)


def test_fused_learner_step_ranking_failure():
    """The one-launch step's ranking giving up (test hook: as a wait of 2^20 polls would, e.g. a
    tile never scheduled) flags its finished envs needs_host = 3 and leaves each at its own
    starting row with next_index unchanged and the sticky failure word set; CurriculumRecord.process
    raises on it; after LearnerEnv.reset_workspace() the launches rank normally."""
    import ctypes
    from acx import _lib
    from acx.agents import CurriculumRecord, LearnerEnv
    L, B, N, H = 36, 2048, 6000, 2
    init = _ms_states(L, N)
    env = LearnerEnv(init, B, horizon_length=H, device=DEV)
    rec = CurriculumRecord(N, B, 0.5)
    hook = _lib.load().acx_internal_learner_ranking_fails
    hook.argtypes = [ctypes.c_int32]
    hook.restype = None
    g = torch.Generator(device=DEV)
    g.manual_seed(7)
    acts = lambda: torch.randint(0, 12, (B,), dtype=torch.int64, device=DEV, generator=g)  # noqa: E731
    env.step(acts())
    hook(1)
    try:
        done, trunc, _, nh = env.step(acts())  # every env truncates at H = 2
    finally:
        hook(0)
    fin = (done | trunc).bool()
    assert bool(fin.all())
    assert bool((nh == 3).all())
    assert torch.equal(env.state, torch.as_tensor(init[:B]).to(DEV))  # own starting rows
    assert int(env.next_index.item()) == B and bool((env.vec.step_count == 0).all())
    assert env.failed()
    with pytest.raises(RuntimeError):
        rec.process(env, done, trunc, nh)
    env.reset_workspace()
    assert not env.failed() and int(env.next_index.item()) == B
    env.step(acts())
    done, trunc, _, nh = env.step(acts())  # all truncate again: ranked normally now
    assert bool((nh == 0).all()) and int(env.next_index.item()) == 2 * B
    assert torch.equal(env.curr_index, torch.arange(B, 2 * B, dtype=torch.int32, device=DEV))
    assert torch.equal(env.state, torch.as_tensor(init[B: 2 * B]).to(DEV))


def test_fused_learner_step_last_total_failure():
    """only the last tile's wait for the batch total gives up (test hook 2).  Every
    tile still ranks its finished envs (they take states B..2B-1), but next_index is stale: the
    launch sets the sticky failure word, CurriculumRecord.process raises, and later launches rank
    nothing (needs_host 3, envs at their own starting rows) until LearnerEnv.reset_workspace()
    re-zeroes the workspace and restores next_index from curr_index; then ranking resumes with
    state 2B, so no initial state is handed out twice."""
    import ctypes
    from acx import _lib
    from acx.agents import CurriculumRecord, LearnerEnv
    L, B, N, H = 36, 2048, 9000, 2
    init = _ms_states(L, N)
    env = LearnerEnv(init, B, horizon_length=H, device=DEV)
    rec = CurriculumRecord(N, B, 0.5)
    hook = _lib.load().acx_internal_learner_ranking_fails
    hook.argtypes = [ctypes.c_int32]
    hook.restype = None
    g = torch.Generator(device=DEV)
    g.manual_seed(11)
    acts = lambda: torch.randint(0, 12, (B,), dtype=torch.int64, device=DEV, generator=g)  # noqa: E731
    env.step(acts())
    hook(2)
    try:
        done, trunc, _, nh = env.step(acts())  # every env truncates at H = 2
    finally:
        hook(0)
    assert bool((done | trunc).bool().all()) and bool((nh == 0).all())
    assert torch.equal(env.curr_index, torch.arange(B, 2 * B, dtype=torch.int32, device=DEV))
    assert torch.equal(env.state, torch.as_tensor(init[B: 2 * B]).to(DEV))
    assert int(env.next_index.item()) == B  # stale: the total never arrived
    assert env.failed()
    with pytest.raises(RuntimeError):
        rec.process(env, done, trunc, nh)
    env.step(acts())
    done, trunc, _, nh = env.step(acts())  # truncate again: nothing is ranked now
    assert bool((nh == 3).all()) and int(env.next_index.item()) == B
    assert torch.equal(env.state, torch.as_tensor(init[B: 2 * B]).to(DEV))
    env.reset_workspace()
    assert not env.failed() and int(env.next_index.item()) == 2 * B
    env.step(acts())
    done, trunc, _, nh = env.step(acts())
    assert bool((nh == 0).all()) and int(env.next_index.item()) == 3 * B
    assert torch.equal(env.curr_index, torch.arange(2 * B, 3 * B, dtype=torch.int32, device=DEV))
    assert torch.equal(env.state, torch.as_tensor(init[2 * B: 3 * B]).to(DEV))
