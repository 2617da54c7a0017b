"""Skeleton graphs (``graph/``): ``ntu_rgb_d`` (25 joints) and ``mediapipe_pose`` (33)."""
