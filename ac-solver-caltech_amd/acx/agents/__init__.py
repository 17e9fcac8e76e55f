"""PPO-side plumbing for the device env (ac_solver/agents/training.py rollout phase)."""
from .curriculum import CurriculumRecord
from .rollout import LearnerEnv

__all__ = ["LearnerEnv", "CurriculumRecord"]
