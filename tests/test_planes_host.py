"""CPU: the bit-plane word algebra of the env-step kernels (ac-solver-caltech_amd/csrc/acx_planes.h,
built for the host) against the C oracle (oracle/acx_oracle.c, itself pinned to the reference's
fixtures by tests/test_oracle.py): ac_move on arbitrary states incl. unreduced words, empty
relators and bad move ids, ac_move_clean on clean states, 200-step walks of clean cyclic moves,
strict triviality and the int8 -> plane pack, at L = 1..64 (one plane word) and 65..128 (two)."""
import os
import subprocess

import pytest

from conftest import PKG_ROOT, REPO

CLANG = "/opt/rocm/lib/llvm/bin/clang"


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    if not os.path.exists(CLANG + "++"):
        pytest.skip("ROCm clang not found")
    d = tmp_path_factory.mktemp("planes")
    obj, exe = str(d / "oracle.o"), str(d / "planes_check")
    subprocess.check_call([CLANG, "-O2", "-c", os.path.join(REPO, "oracle", "acx_oracle.c"), "-o", obj])
    subprocess.check_call([CLANG + "++", "-O2", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-DACX_PLANES_HOST_CHECK",
                           "-I/opt/rocm/include", "-I", os.path.join(REPO, "include"), "-I",
                           os.path.join(PKG_ROOT, "csrc"), os.path.join(REPO, "tests", "planes_check.cpp"), obj,
                           "-o", exe])
    return exe


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_planes_algebra_matches_oracle(checker, seed):
    r = subprocess.run([checker, "20000", str(seed)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stdout[-2000:]
