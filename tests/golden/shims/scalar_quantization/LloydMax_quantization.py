"""A13: scalar_quantization.LloydMax_quantization (un-vendored), restated as the
textbook Lloyd-Max design over the integer histogram it is given.

  L = max_val - min_val + 1 histogram bins (value v = min_val + i), N = ceil(L / Q_step)
  cells; cell j holds the bins [lo_j, lo_{j+1}), starting from the uniform cells
  lo_j = j Q_step (lo_N = L).  One iteration: centroid c_j = sum(v n_v) / sum(n_v)
  over the cell (exact int64 sums, one float64 division), then lo_j = ceil((c_{j-1}
  + c_j) / 2) - min_val for j = 1..N-1; stop when the cells do not change (at most
  100 iterations); the centroids of the final cells are the representation levels.
  encode(x) = number of thresholds (c_{j-1} + c_j) / 2 that are <= x
  (searchsorted 'right', float64 comparison); decode(k) = centroids[k].
Unpinned (the package is not in this image).
"""
import math

import numpy as np

name = "LloydMax"
MAX_ITERS = 100


class LloydMax_Quantizer:
    def __init__(self, Q_step, counts, min_val=0, max_val=255):
        self.Q_step = int(Q_step)
        self.min_val, self.max_val = int(min_val), int(max_val)
        counts = np.asarray(counts).astype(np.int64)
        # the decoder builds a throw-away quantizer from np.ones(L) without the
        # range (LloydMax.py:140) and then sets the levels: the histogram's
        # length defines the bins
        L = counts.shape[0]
        self.max_val = self.min_val + L - 1
        N = -(-L // self.Q_step)
        v = np.arange(self.min_val, self.max_val + 1, dtype=np.int64)
        S0 = np.concatenate([[0], np.cumsum(counts)])
        S1 = np.concatenate([[0], np.cumsum(counts * v)])

        def centroids(lo):
            return np.array([float(S1[lo[j + 1]] - S1[lo[j]]) / float(S0[lo[j + 1]] - S0[lo[j]])
                             for j in range(N)], np.float64)

        lo = [j * self.Q_step for j in range(N)] + [L]
        for _ in range(MAX_ITERS):
            c = centroids(lo)
            new = [0] + [math.ceil((c[j - 1] + c[j]) / 2) - self.min_val for j in range(1, N)] + [L]
            if new == lo:
                break
            lo = new
        self.set_representation_levels(centroids(lo))

    def get_representation_levels(self):
        return self.centroids.copy()

    def set_representation_levels(self, centroids):
        self.centroids = np.asarray(centroids, np.float64)
        self.thresholds = (self.centroids[:-1] + self.centroids[1:]) / 2

    def encode(self, x):
        return np.searchsorted(self.thresholds, x, side="right")

    def decode(self, k):
        return self.centroids[k]
