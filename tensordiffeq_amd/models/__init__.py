"""Solver API (reference layer L6: tensordiffeq/models.py) and networks (L3)."""
from . import networks
from .networks import TanhMLP, FlatModule, neural_net
from .collocation import CollocationSolverND
from .discovery import DiscoveryModel, Variable

__all__ = ["networks", "TanhMLP", "FlatModule", "neural_net", "CollocationSolverND", "DiscoveryModel", "Variable"]
