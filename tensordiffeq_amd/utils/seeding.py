"""Global seeding.  The reference is unseeded (B21); here every random draw (LHS, BC subsets,
network init) goes through one seedable source so runs and DP ranks are reproducible."""
from __future__ import annotations

import numpy as np
import torch

_STATE = {"seed": None, "np": np.random.RandomState()}


def set_seed(seed):
    _STATE["seed"] = int(seed)
    _STATE["np"] = np.random.RandomState(int(seed))
    torch.manual_seed(int(seed))


def numpy_rng():
    return _STATE["np"]


def current_seed():
    return _STATE["seed"]
