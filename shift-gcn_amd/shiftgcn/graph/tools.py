"""Adjacency helpers (``graph/tools.py``). The Shift-GCN compute path never reads ``A``
(``Shift_gcn`` ignores it, shift_gcn.py:78-142); it is built only so that ``Model`` keeps
the reference constructor contract (``graph`` dotted path -> ``Graph(**graph_args).A``)."""
import numpy as np


def edge2mat(link, num_node):
    A = np.zeros((num_node, num_node))
    for i, j in link:
        A[j, i] = 1
    return A


def normalize_digraph(A):
    """Column-normalise: A @ diag(1 / column sums) (zero columns stay zero)."""
    col = A.sum(0)
    inv = np.where(col > 0, 1.0 / np.where(col > 0, col, 1.0), 0.0)
    return A * inv[None, :]


def get_spatial_graph(num_node, self_link, inward, outward):
    return np.stack((edge2mat(self_link, num_node),
                     normalize_digraph(edge2mat(inward, num_node)),
                     normalize_digraph(edge2mat(outward, num_node))))


class SkeletonGraph:
    num_node = 0
    inward = ()

    def __init__(self, labeling_mode="spatial"):
        n = self.num_node
        self.self_link = [(i, i) for i in range(n)]
        self.inward = list(type(self).inward)
        self.outward = [(j, i) for (i, j) in self.inward]
        self.neighbor = self.inward + self.outward
        if labeling_mode != "spatial":
            raise ValueError()
        self.A = get_spatial_graph(n, self.self_link, self.inward, self.outward)

    def get_adjacency_matrix(self, labeling_mode=None):
        return self.A
