"""Optimizers (reference layer L4: tensordiffeq/optimizers.py + Keras Adam)."""
from .adam import Adam, torch_update, bias_corrected_lr
from .lbfgs import eager_lbfgs, graph_lbfgs, LBFGSWolfe, Struct, dot, compact_direction
from . import lbfgs_device
from .lbfgs_device import DeviceLBFGS

__all__ = ["Adam", "torch_update", "bias_corrected_lr", "eager_lbfgs", "graph_lbfgs",
           "LBFGSWolfe", "Struct", "dot", "compact_direction", "lbfgs_device", "DeviceLBFGS"]
