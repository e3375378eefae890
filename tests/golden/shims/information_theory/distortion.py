"""A7: RMSE as computed in-tree by src/RDE.py:40-53."""
import numpy as np


def RMSE(x, y):
    return float(np.sqrt(np.mean((x.astype(np.float64) - y) ** 2)))
