"""Error metrics (reference tensordiffeq/helpers.py:3-4)."""
from __future__ import annotations

import numpy as np


def find_L2_error(u_pred, u_star):
    """Relative L2 error ||u* - u||_2 / ||u*||_2."""
    u_pred = np.asarray(u_pred, dtype=np.float64).reshape(-1)
    u_star = np.asarray(u_star, dtype=np.float64).reshape(-1)
    return float(np.linalg.norm(u_star - u_pred, 2) / np.linalg.norm(u_star, 2))
