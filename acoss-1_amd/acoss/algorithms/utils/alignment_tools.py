"""Constrained Smith-Waterman (acoss/algorithms/utils/alignment_tools.py) on the HIP engine.

`smith_waterman_constrained` keeps the reference's signature (one binary matrix -> float);
`smith_waterman_constrained_batch` scores a list of matrices in one launch (one wavefront
per matrix, misc.hip k_sw). Non-binary input raises IOError like `match` (:17-23).
"""
import numpy as np

from ... import _lib

__all__ = ["smith_waterman_constrained", "smith_waterman_constrained_batch"]


def smith_waterman_constrained_batch(mats):
    return _lib.sw_constrained(list(mats)).cpu().numpy()


def smith_waterman_constrained(input_matrix):
    """Max of the constrained local-alignment score matrix (alignment_tools.py:27-46)."""
    return float(smith_waterman_constrained_batch([np.asarray(input_matrix)])[0])
