"""Numerics utilities (reference layer L1: tensordiffeq/utils.py)."""
from .mesh import multimesh, flatten_and_stack
from .numerics import (MSE, g_MSE, constant, convertTensor, tensor, get_tf_model, get_model,
                       get_sizes, get_weights, set_weights, initialize_weights_loss, DEFAULT_DTYPE)
from .seeding import set_seed, numpy_rng, current_seed
from . import seeding


def LatinHypercubeSample(N_f, bounds, criterion="c", random_state=None):
    from ..sampling import LatinHypercubeSample as _lhs
    return _lhs(N_f, bounds, criterion=criterion, random_state=random_state)


__all__ = ["multimesh", "flatten_and_stack", "MSE", "g_MSE", "constant", "convertTensor", "tensor",
           "get_tf_model", "get_model", "get_sizes", "get_weights", "set_weights",
           "initialize_weights_loss", "LatinHypercubeSample", "set_seed", "numpy_rng",
           "current_seed", "DEFAULT_DTYPE"]
