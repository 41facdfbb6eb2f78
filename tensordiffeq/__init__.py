"""Import alias: ``import tensordiffeq as tdq`` resolves to :mod:`tensordiffeq_amd`.

Lets scripts written against the reference's module layout (``tensordiffeq.models``,
``tensordiffeq.boundaries``, ``tensordiffeq.utils`` ...) import this framework unchanged; every
submodule name maps to the same module object of ``tensordiffeq_amd``.
"""
import importlib
import sys

import tensordiffeq_amd as _impl

_SUBMODULES = ["models", "optimizers", "plotting", "utils", "domains", "boundaries", "fit",
               "helpers", "sampling", "output", "checkpoint", "parallel", "ops", "jet", "autodiff"]

for _name in _SUBMODULES:
    sys.modules[f"{__name__}.{_name}"] = importlib.import_module(f"tensordiffeq_amd.{_name}")
sys.modules[f"{__name__}.networks"] = _impl.models.networks

from tensordiffeq_amd import *  # noqa: E402,F401,F403
from tensordiffeq_amd import __all__, __version__  # noqa: E402,F401

networks = _impl.models.networks
