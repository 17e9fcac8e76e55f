"""GPU: bench.py end to end at a small batch, in a child process (as the driver runs it): one
JSON line with the contract's fields, the rollout split into launches of <= 200 steps through
ops.RolloutPlan (K = 210: a packed 200-step launch and a direct-id 10-step one), no env
errors, and the roofline / variant blocks present."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=240, env=None):
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], cwd=REPO, capture_output=True,
                       text=True, timeout=timeout, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout[-3000:]
    return json.loads(lines[0])


def test_bench_line_multi_launch_small_batch():
    d = _bench("--batch", "8192", "--steps", "210", "--warmup", "3", "--no-cpu", "--no-bfs", "--no-learner",
               "--no-graph", "--no-search")
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 210 and d["warmup"] == 3
    assert d["value"] > 0 and d["env_errors"] == 0
    r = d["roofline"]
    assert r["launches"] == 2 and r["kernel"].startswith("acx::pack_actions_kernel")
    assert 0 < r["frac"] < 1.5 and r["bytes_per_env_step"] == 298
    assert d["config"]["envs_per_gpu"] == 8192
    for v in ("rollout_obs_int8", "rollout_desync", "step_api"):
        assert v in d["variants"] and d["variants"][v].get("env_errors", 0) == 0, v


def test_bench_line_short_launch_reads_int32_ids():
    d = _bench("--batch", "4096", "--steps", "20", "--warmup", "5", "--no-cpu", "--no-bfs", "--no-learner",
               "--no-graph", "--no-step-api", "--no-desync", "--no-obs8", "--no-search")
    r = d["roofline"]
    assert r["launches"] == 1 and r["kernel"].startswith("acx::rollout_kernel")
    assert d["env_errors"] == 0 and d["value"] > 0


def test_bench_step_workload_headline():
    # config 5's shape (--workload step) at a small batch: the per-call step API is the headline
    # (the lengths-carrying acx_step_lengths; acx_step on the same walk is a variant)
    d = _bench("--workload", "step", "--L", "128", "--batch", "8192", "--steps", "12", "--warmup", "2", "--no-cpu",
               "--no-bfs", "--no-learner", "--no-search")
    assert d["n_gpus"] == 1 and d["world_size_seen"] == 1 and d["env_errors"] == 0
    assert d["roofline"]["kernel"] == "acx::step_lengths_kernel<8,128,4>" and d["roofline"]["launches"] == 12
    v = d["variants"]
    assert v["step_api"]["roofline"]["kernel"] == "acx::step_kernel<8,128,4,false>"
    assert v["step_api_lengths"]["same_states_as_step_api"] and v["step_api_lengths"]["env_errors"] == 0
    assert "random-action stepping" in d["config"]["workload"]
    assert "rollout_obs_int8" not in d["variants"] and "step_api_hipgraph" in d["variants"]
    r8 = d["variants"]["stepping_rollout_obs_int8"]
    assert r8["env_errors"] == 0 and r8["value"] > 0 and r8["roofline"]["kernel"] == "acx::rollout_kernel<8,128,4,2>"


def test_bench_launcher_two_ranks_gloo_one_gpu():
    # bench.py --gpus 2 starts both ranks itself; gloo puts both on cuda:0 (one-GPU box)
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                                            "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env["ACX_DIST_BACKEND"] = "gloo"
    d = _bench("--gpus", "2", "--batch", "8192", "--steps", "20", "--warmup", "5", "--no-cpu", "--no-bfs",
               "--no-learner", "--no-graph", "--no-step-api", "--no-desync", "--no-obs8", env=env)
    assert d["n_gpus"] == 2 and d["world_size_seen"] == 2 and d["dist_backend"] == "gloo"
    assert len(d["per_rank"]) == 2 and all(r["value"] > 0 for r in d["per_rank"])
    assert d["config"]["global_batch"] == 2 * 8192 and d["env_errors"] == 0
