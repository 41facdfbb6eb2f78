"""Optimizers (reference layer L4: tensordiffeq/optimizers.py + Keras Adam)."""
from .adam import Adam, torch_update, bias_corrected_lr
from .lbfgs import eager_lbfgs, graph_lbfgs, LBFGSWolfe, Struct, dot, compact_direction

__all__ = ["Adam", "torch_update", "bias_corrected_lr", "eager_lbfgs", "graph_lbfgs",
           "LBFGSWolfe", "Struct", "dot", "compact_direction"]
