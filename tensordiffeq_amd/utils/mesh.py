"""Tensor-product mesh helpers used to build boundary / initial-condition point sets.

Behavioural parity with the reference helpers ``multimesh`` and ``flatten_and_stack``
(reference: tensordiffeq/utils.py:72-99): ``multimesh`` returns one array per input axis,
broadcast to the full product shape in ``ij`` order, and ``flatten_and_stack`` turns those
arrays into an ``(n_points, n_axes)`` matrix.  Implemented with ``np.meshgrid`` instead of
the reference's repeat loops.
"""
from __future__ import annotations

import numpy as np


def multimesh(arrs):
    """Return ``len(arrs)`` arrays of shape ``(len(a0), len(a1), ...)`` (``ij`` indexing)."""
    arrs = [np.asarray(a).reshape(-1) for a in arrs]
    if not arrs:
        return []
    return list(np.meshgrid(*arrs, indexing="ij"))


def flatten_and_stack(mesh):
    """Stack flattened mesh arrays column-wise into an ``(n_points, n_axes)`` float64 matrix."""
    if len(mesh) == 0:
        return np.zeros((1, 0))
    return np.stack([np.asarray(m, dtype=np.float64).reshape(-1) for m in mesh], axis=1)
