"""NTU RGB+D 25-joint skeleton (``graph/ntu_rgb_d.py``)."""
from .tools import SkeletonGraph

num_node = 25
_edges_1based = [(1, 2), (2, 21), (3, 21), (4, 3), (5, 21), (6, 5), (7, 6), (8, 7), (9, 21),
                 (10, 9), (11, 10), (12, 11), (13, 1), (14, 13), (15, 14), (16, 15), (17, 1),
                 (18, 17), (19, 18), (20, 19), (22, 23), (23, 8), (24, 25), (25, 12)]


class Graph(SkeletonGraph):
    num_node = num_node
    inward = [(i - 1, j - 1) for (i, j) in _edges_1based]
