from .breadth_first import bfs
from .greedy import greedy_search

__all__ = ["bfs", "greedy_search"]
