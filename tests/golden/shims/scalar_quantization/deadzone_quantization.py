"""A5: deadzone quantizer, truncation toward zero, mid-tread reconstruction Q*k."""
import numpy as np

name = "deadzone"


class Deadzone_Quantizer:
    def __init__(self, Q_step, min_val=-128, max_val=127):
        self.Q_step = Q_step
        self.min_val, self.max_val = min_val, max_val

    def encode(self, x):
        return (x / self.Q_step).astype(np.int32)

    def decode(self, k):
        return self.Q_step * k
