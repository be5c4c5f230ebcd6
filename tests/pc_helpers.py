"""Test helpers (path cache handle lives in shadow-1_amd/sim.py)."""
import numpy as np

from sim import PathCache, SHD_PC_FORCE_ROWS  # noqa: F401


def same_bits(a, b):
    """Bitwise equality of f64 arrays (NaN == NaN with the same payload)."""
    a = np.ascontiguousarray(a, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64)
    return a.shape == b.shape and np.array_equal(a.view(np.uint64), b.view(np.uint64))
