"""acx -- MI355X-native Andrews-Curtis environment (the ACEnv.step / 12-way expansion hot
path of Avi161/AC-Solver-Caltech), HIP kernels behind the C-ABI in include/acx.h.

Public names mirror the reference's ac_solver/__init__.py:1-6 (ACEnv, ACEnvConfig, bfs,
greedy_search); VecACEnv and acx.ops are the batched device API.
"""

from .envs.ac_env import ACEnv, ACEnvConfig, VecACEnv
from .envs.ac_moves import ACMove
from .search.breadth_first import bfs
from .search.greedy import greedy_search
from . import data  # noqa: F401

__all__ = ["ACEnv", "ACEnvConfig", "VecACEnv", "ACMove", "bfs", "greedy_search"]
