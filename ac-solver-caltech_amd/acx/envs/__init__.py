from .ac_env import ACEnv, ACEnvConfig, VecACEnv
from .ac_moves import ACMove

__all__ = ["ACEnv", "ACEnvConfig", "VecACEnv", "ACMove"]
