"""Minimal stand-ins for the gym 0.10.9 spaces the reference exposes
(requirements.txt:32; multi_discrete.py SOURCES.txt:16). gym is not a
dependency of this package; only the attributes runners read are provided."""
from __future__ import annotations

import numpy as np


class Discrete:
    def __init__(self, n: int):
        self.n = int(n)
        self.shape = ()
        self.dtype = np.int64

    def __repr__(self):
        return f"Discrete({self.n})"


class Box:
    def __init__(self, low, high, shape, dtype=np.float32):
        self.low, self.high = low, high
        self.shape = tuple(shape)
        self.dtype = dtype

    def __repr__(self):
        return f"Box({self.shape})"
