"""Host code under the compiler's sanitizers ("Race detection / sanitizers").  CPU
only; each test builds what it runs with g++/gcc into a temporary directory.

* The host-dedup search engine (ac-solver-caltech_amd/csrc/acx_search.cpp: a thread pool, a
  visited set partitioned by hash over the threads, provisional entries that other threads
  finalise) under ThreadSanitizer, and separately under AddressSanitizer + UBSan, at
  ACX_HOST_THREADS = 1, 3 and 16, on
    - the 240 reference bfs / greedy runs of tests/golden/kat_search_extra.json (the
      reference's breadth_first.py:15-97 / greedy.py:15-121, its set-based dedup at
      breadth_first.py:56,87-89), results checked as test_cpu_host.py checks them, and
    - AK(3) to 10^6 nodes (config 4's start; tools/host_bfs_bench.cpp), node / parent counts equal
      at every thread count;
  expansions come from the C oracle (tests/sanitize/search_harness.cpp), so no GPU is involved.
* The C oracle itself (oracle/Makefile liboracle_asan.so, ASan + UBSan): tests/test_oracle.py
  run against it.
Any sanitizer report fails the test (halt_on_error, and the report text is searched for)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import GOLDEN, REPO

CSRC = os.path.join(REPO, "ac-solver-caltech_amd", "csrc")
REPORT_MARKERS = ("WARNING: ThreadSanitizer", "ERROR: AddressSanitizer", "runtime error:", "ERROR: LeakSanitizer",
                  "SUMMARY: UndefinedBehaviorSanitizer")
SAN_FLAGS = {
    "tsan": ["-fsanitize=thread"],
    "asan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer"],
}
SAN_ENV = {
    "TSAN_OPTIONS": "halt_on_error=1:exitcode=66:second_deadlock_stack=1",
    "ASAN_OPTIONS": "halt_on_error=1:exitcode=66:detect_leaks=1",
    "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1:exitcode=66",
}


def _build(kind, main_src, out):
    cmd = (["g++", "-O1", "-g", "-std=c++17", "-pthread"] + SAN_FLAGS[kind] +
           ["-I" + os.path.join(REPO, "include"), main_src, os.path.join(CSRC, "acx_search.cpp"),
            "-x", "c", os.path.join(REPO, "oracle", "acx_oracle.c"), "-o", out])
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return out


def _run(exe, args=(), stdin=None, threads="1", timeout=600):
    env = dict(os.environ, ACX_HOST_THREADS=threads, **SAN_ENV)
    r = subprocess.run([exe, *args], input=stdin, capture_output=True, text=True, env=env, timeout=timeout)
    reports = [m for m in REPORT_MARKERS if m in r.stderr]
    assert r.returncode == 0 and not reports, (exe, threads, r.returncode, reports, r.stderr[-4000:])
    return r.stdout


@pytest.fixture(scope="module", params=["tsan", "asan"])
def harness(request, tmp_path_factory):
    d = tmp_path_factory.mktemp(request.param)
    return request.param, _build(request.param, os.path.join(REPO, "tests", "sanitize", "search_harness.cpp"),
                                 str(d / "search_harness"))


@pytest.mark.slow
@pytest.mark.parametrize("threads", ["1", "3", "16"])
def test_search_engine_sanitized_on_reference_runs(harness, threads):
    kind, exe = harness
    with open(os.path.join(GOLDEN, "kat_search_extra.json")) as f:
        cases = json.load(f)
    lines = []
    for c in cases:
        p = c["presentation"]
        mode = 0 if c["search_fn"] == "bfs" else 1
        lines.append(f"{mode} {len(p) // 2} {int(c['cyclical'])} {c['budget']} " + " ".join(map(str, p)))
    out = _run(exe, stdin="\n".join(lines) + "\n", threads=threads).strip().split("\n")
    assert len(out) == len(cases)
    for c, line in zip(cases, out):
        v = [int(x) for x in line.split()]
        status, n_nodes, m = v[0], v[1], v[2]
        path = [(v[3 + 2 * i], v[4 + 2 * i]) for i in range(m)]
        if c["raises"]:
            assert status == 3, c
            continue
        assert status in (1, 2), c
        assert (status == 1) == c["ok"], c
        if c["search_fn"] == "bfs":
            assert (path if status == 1 else None) == (None if c["path"] is None else [tuple(x) for x in c["path"]]), c
        else:
            assert path == [tuple(x) for x in c["path"]], c
        if c["budget_nodes"] is not None:
            assert n_nodes == c["budget_nodes"], c


@pytest.mark.slow
def test_search_engine_sanitized_ak3_1e6(tmp_path):
    """AK(3) to 10^6 nodes (tools/host_bfs_bench.cpp), both sanitizer builds, 1 / 3 / 16 threads:
    no report, and the same node and parent counts at every thread count."""
    results = {}
    for kind in ("tsan", "asan"):
        exe = _build(kind, os.path.join(REPO, "tools", "host_bfs_bench.cpp"), str(tmp_path / f"bfs_{kind}"))
        for threads in ("1", "3", "16"):
            out = _run(exe, [str(10 ** 6), str(tmp_path / "children.bin")], threads=threads)
            rec = json.loads(out.strip().split("\n")[-1])
            results[(kind, threads)] = (rec["status"], rec["budget"], rec["nodes"], rec["parents"])
    assert len(set(results.values())) == 1, results
    status, budget, nodes, parents = next(iter(results.values()))
    assert status == 2 and budget == 1 and nodes >= 10 ** 6, results


@pytest.mark.slow
def test_oracle_under_asan_ubsan(tmp_path):
    """tests/test_oracle.py (every reference fixture) against oracle/liboracle_asan.so, in a child
    Python with the ASan runtime preloaded (the interpreter itself is not instrumented)."""
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "liboracle_asan.so"], check=True)
    asan_rt = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True,
                             check=True).stdout.strip()
    env = dict(os.environ, LD_PRELOAD=asan_rt, ACX_ORACLE_LIB=os.path.join(REPO, "oracle", "liboracle_asan.so"),
               ASAN_OPTIONS="halt_on_error=1:exitcode=66:detect_leaks=0", UBSAN_OPTIONS=SAN_ENV["UBSAN_OPTIONS"])
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        os.path.join(REPO, "tests", "test_oracle.py")], capture_output=True, text=True, env=env,
                       cwd=str(tmp_path), timeout=900)
    reports = [m for m in REPORT_MARKERS if m in r.stdout + r.stderr]
    assert r.returncode == 0 and not reports, (r.returncode, reports, r.stdout[-3000:], r.stderr[-3000:])
    assert " passed" in r.stdout
