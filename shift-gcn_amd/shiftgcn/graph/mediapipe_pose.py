"""MediaPipe Pose 33-landmark skeleton (``graph/mediapipe_pose.py``): a spanning tree
rooted at the nose, edges (child, parent)."""
from .tools import SkeletonGraph

num_node = 33


class Graph(SkeletonGraph):
    num_node = num_node
    inward = [(1, 0), (2, 1), (3, 2), (7, 3), (4, 0), (5, 4), (6, 5), (8, 6), (9, 0), (10, 9),
              (11, 0), (12, 11), (13, 11), (15, 13), (17, 15), (19, 15), (21, 15), (14, 12),
              (16, 14), (18, 16), (20, 16), (22, 16), (23, 11), (24, 12), (25, 23), (27, 25),
              (29, 27), (31, 27), (26, 24), (28, 26), (30, 28), (32, 28)]
