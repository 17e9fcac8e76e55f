"""CPU: bench.py's multi-rank launcher and its checks, with no GPU (`--dry-run`: gloo, a numpy pass
per step in place of the kernels).

* `bench.py --gpus 2` with no torchrun environment starts two rank processes itself, both join one
  process group, and rank 0 prints ONE line with n_gpus 2, world_size_seen 2 and a per-rank block;
* a torchrun group whose size differs from --gpus fails with a non-zero status (no line);
* a rank that fails makes the launcher fail with that rank's status;
* every line carries the CPU baselines, N > 1 included (measured by the launcher before it starts
  the ranks, or by rank 0 before it joins the process group under torchrun)."""
import json
import os
import socket
import subprocess
import sys

from conftest import REPO

BENCH = os.path.join(REPO, "bench.py")


def _env():
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def _lines(out):
    return [json.loads(x) for x in out.splitlines() if x.startswith("{")]


def test_launcher_spawns_two_ranks_one_line():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run", "--steps", "4", "--warmup", "1",
                        "--batch", "512", "--no-cpu"], cwd=REPO, capture_output=True, text=True, timeout=180, env=_env())
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _lines(p.stdout)
    assert len(lines) == 1, p.stdout
    d = lines[0]
    assert d["n_gpus"] == 2 and d["world_size_seen"] == 2 and d["dry_run"] is True
    assert [r["rank"] for r in d["per_rank"]] == [0, 1]
    assert d["config"]["global_batch"] == 1024 and d["config"]["envs_per_gpu"] == 512
    # value = all ranks' env-steps / max-over-ranks wall time
    assert abs(d["value"] - 2 * 512 * 4 / (d["ms_per_step"] * 4 / 1e3)) < 1e-6 * d["value"]


def test_one_rank_line_has_the_same_shape():
    p = subprocess.run([sys.executable, BENCH, "--dry-run", "--steps", "3", "--warmup", "0", "--batch", "256", "--no-cpu"],
                       cwd=REPO, capture_output=True, text=True, timeout=120, env=_env())
    assert p.returncode == 0, p.stderr[-3000:]
    (d,) = _lines(p.stdout)
    assert d["n_gpus"] == 1 and d["world_size_seen"] == 1 and len(d["per_rank"]) == 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_world_size_mismatch_fails():
    # torchrun starts 2 ranks but the command says --gpus 3: every rank refuses to measure
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), BENCH, "--gpus", "3",
                        "--dry-run", "--steps", "2", "--warmup", "0", "--batch", "64", "--no-cpu"],
                       cwd=REPO, capture_output=True, text=True, timeout=180, env=_env())
    assert p.returncode != 0
    assert not _lines(p.stdout)
    assert "process group has 2 rank(s), --gpus 3" in p.stderr


def test_failing_rank_fails_the_launcher():
    sys.path.insert(0, REPO)
    import bench

    # every rank rejects the argument list (argparse exits 2); the launcher returns that status
    rc = bench.spawn_ranks(2, ["--dry-run", "--workload", "no-such-workload"])
    assert rc == 2


_GUARD = """
import os, signal, sys, time
sys.path.insert(0, {repo!r})
import bench
line = {{"metric": "m", "value": 1.0, "variants": {{}}}}
with bench.LineGuard(line, line["variants"], "sharded_bfs", 0, {timeout}):
    if {kill}:
        os.kill(os.getpid(), signal.SIGTERM)
    time.sleep({sleep})  # the main thread inside a C call, as in an RCCL wait
print("left the guard")
"""


def _guard(timeout, kill, sleep):
    code = _GUARD.format(repo=REPO, timeout=timeout, kill=kill, sleep=sleep)
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)


def test_line_guard_prints_the_line_when_torchrun_stops_the_rank():
    """SIGTERM (torchrun's stop of the surviving ranks) while the main thread is blocked: the line
    is printed with the variant marked and the process exits EXIT_BFS_STALL, long before the sleep
    or the deadline would end."""
    p = _guard(30.0, True, 20)
    assert p.returncode == 3, (p.returncode, p.stderr[-2000:])
    lines = _lines(p.stdout)
    assert len(lines) == 1 and "left the guard" not in p.stdout
    assert lines[0]["value"] == 1.0 and "SIGTERM" in lines[0]["variants"]["sharded_bfs"]["error"]


def test_line_guard_deadline():
    p = _guard(0.5, False, 20)
    assert p.returncode == 3, (p.returncode, p.stderr[-2000:])
    lines = _lines(p.stdout)
    assert len(lines) == 1 and "timeout" in lines[0]["variants"]["sharded_bfs"]["error"]


def test_line_guard_disarms_on_exit():
    p = _guard(30.0, False, 0.2)
    assert p.returncode == 0, p.stderr[-2000:]
    assert _lines(p.stdout) == [] and "left the guard" in p.stdout


def test_strong_scaling_splits_the_global_batch():
    """--global-batch: the total is fixed and split over the ranks (SURVEY 8(d) strong scaling)."""
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run", "--steps", "3", "--warmup", "1",
                        "--global-batch", "1024", "--no-cpu"], cwd=REPO, capture_output=True, text=True, timeout=180, env=_env())
    assert p.returncode == 0, p.stderr[-3000:]
    (d,) = _lines(p.stdout)
    assert d["scaling"] == "strong" and d["n_gpus"] == 2
    assert d["config"]["global_batch"] == 1024 and d["config"]["envs_per_gpu"] == 512
    bad = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run", "--global-batch", "1000", "--no-cpu"], cwd=REPO,
                         capture_output=True, text=True, timeout=180, env=_env())
    assert bad.returncode != 0 and "multiple of 64" in bad.stderr


def _check_cpu(d, where):
    for k in ("cpu_baseline", "cpu_baseline_c_oracle", "cpu_baseline_c_oracle_all_cores"):
        c = d[k]
        assert c and c["value"] > 0 and c["cores"] >= 1 and c["unit"] == "env-steps/s", k
        assert where in c["measured"], (k, c["measured"])
    assert d["cpu_baseline"]["kind"] == "port"


def test_launcher_line_carries_cpu_baseline():
    """`bench.py --gpus 2` (the launcher) puts the CPU baselines -- measured on
    the host's cores before any rank started -- into rank 0's line."""
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run", "--steps", "2", "--warmup", "0",
                        "--batch", "256", "--cpu-seconds", "1"], cwd=REPO, capture_output=True, text=True,
                       timeout=240, env=_env())
    assert p.returncode == 0, p.stderr[-3000:]
    (d,) = _lines(p.stdout)
    assert d["n_gpus"] == 2
    _check_cpu(d, "launcher")


def test_torchrun_line_carries_cpu_baseline():
    """Under torchrun (the driver's N > 1 command) rank 0 measures the CPU baselines before it joins
    the process group."""
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), BENCH, "--gpus", "2",
                        "--dry-run", "--steps", "2", "--warmup", "0", "--batch", "256", "--cpu-seconds", "1"],
                       cwd=REPO, capture_output=True, text=True, timeout=240, env=_env())
    assert p.returncode == 0, p.stderr[-3000:]
    (d,) = _lines(p.stdout)
    assert d["n_gpus"] == 2
    _check_cpu(d, "rank 0 of 2")
