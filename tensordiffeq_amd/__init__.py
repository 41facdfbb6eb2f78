"""tensordiffeq_amd - collocation PINNs on AMD MI355X (PyTorch-ROCm + HIP/CDNA4 kernels + RCCL).

Public API mirrors TensorDiffEq (reference tensordiffeq/__init__.py + the re-exports older builds
had): ``DomainND``, the BC/IC classes, ``CollocationSolverND``, ``DiscoveryModel``, utilities,
plotting and helpers.  Derivatives inside user residuals use :func:`grad` (``tf.gradients``-style
:func:`gradients` also provided).
"""
from . import utils, sampling, domains, boundaries, autodiff, jet, helpers, plotting, output
from . import optimizers, parallel, ops, checkpoint, fit
from . import models
from .autodiff import grad, gradients
from .domains import DomainND
from .boundaries import dirichletBC, FunctionDirichletBC, FunctionNeumannBC, IC, periodicBC
from .models import CollocationSolverND, DiscoveryModel, TanhMLP, neural_net, Variable
from .utils import (constant, tensor, convertTensor, LatinHypercubeSample, MSE, g_MSE, set_seed,
                    multimesh, flatten_and_stack)
from .helpers import find_L2_error
from .plotting import newfig, get_griddata
from .parallel import init_distributed

networks = models.networks

__version__ = "0.2.0"

from . import config, metrics, profiling  # noqa: E402
from .config import SolverConfig  # noqa: E402

__all__ = ["models", "networks", "plotting", "utils", "helpers", "optimizers", "boundaries",
           "domains", "fit", "sampling", "parallel", "ops", "checkpoint", "jet", "autodiff",
           "grad", "gradients", "DomainND", "dirichletBC", "FunctionDirichletBC",
           "FunctionNeumannBC", "IC", "periodicBC", "CollocationSolverND", "DiscoveryModel",
           "TanhMLP", "neural_net", "Variable", "constant", "tensor", "convertTensor",
           "LatinHypercubeSample", "MSE", "g_MSE", "set_seed", "multimesh", "flatten_and_stack",
           "find_L2_error", "newfig", "get_griddata", "init_distributed", "config", "metrics",
           "SolverConfig"]
