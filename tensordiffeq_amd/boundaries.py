"""Boundary and initial conditions (reference tensordiffeq/boundaries.py:1-249).

Every condition turns a :class:`DomainND` plus user callables into host point sets
(``(n, ndim)`` float64 arrays, columns in ``domain.vars`` order) and target values.  The solver
moves them to the device once at compile time.

Classes and the reference behaviour they keep:
  dirichletBC          boundaries.py:41-59   u(face) = const
  FunctionDirichletBC  boundaries.py:62-101  u(face) = fun(face coords); optional random subset
  FunctionNeumannBC    boundaries.py:103-156 d_k(u)(face) = fun(...)  (deriv_model callables)
  IC                   boundaries.py:163-203 u(t=t0) = fun(space coords)
  periodicBC           boundaries.py:205-246 d_k(u)(upper face) = d_k(u)(lower face)

Deliberate fixes: ``n_values=None`` works for FunctionDirichletBC (B18); the
time column of ``IC`` is inserted at ``vars.index(time_var)`` instead of appended (B19); the
debug print is gone (B28).  Random face subsets keep the reference's sampling *with*
replacement by default (B20, ``replace=False`` opts out) and draw from the package RNG.
"""
from __future__ import annotations

import numpy as np

from .domains import DomainND
from .utils.mesh import multimesh, flatten_and_stack
from .utils import seeding

import torch  # noqa: E402  (re-exported like the reference leaked ``np``/``tf``)

__all__ = ["BC", "dirichletBC", "FunctionDirichletBC", "FunctionNeumannBC", "IC", "periodicBC",
           "DomainND", "get_linspace", "np", "torch"]


def get_linspace(dict_):
    return [val for key, val in dict_.items() if key.endswith("linspace")][0]


def _subset(n_total, n_values, replace, force=False):
    """Indices of a random face subset (``None`` = keep every point in order)."""
    if n_values is None and not force:
        return None
    size = n_total if n_values is None else int(n_values)
    rng = seeding.numpy_rng()
    if replace:
        return rng.randint(0, n_total, size=size)
    return rng.choice(n_total, size=min(size, n_total), replace=False)


class BC:
    """Base class; subclasses set exactly one of the ``is*`` flags."""

    isPeriodic = False
    isInit = False
    isNeumann = False
    isDirichlect = False  # (sic) reference spelling, kept for user code that checks it

    @property
    def isDirichlet(self):
        return self.isDirichlect

    kind = "bc"

    def get_dict(self, var):
        return self.domain.get_dict(var)

    def _face_mesh(self, var, value):
        """All grid points of the face ``var = value`` (other axes on their linspaces)."""
        others = [v for v in self.domain.vars if v != var]
        mesh = flatten_and_stack(multimesh([self.domain.linspace(v) for v in others]))
        col = np.full((mesh.shape[0],), float(value))
        return np.insert(mesh, self.domain.vars.index(var), col, axis=1)

    def _eval_funs(self, funs, func_inputs):
        vals = []
        for i, names in enumerate(func_inputs):
            if isinstance(names, str):
                names = [names]
            grid = flatten_and_stack(multimesh([self.domain.linspace(v) for v in names]))
            out = funs[i](*grid.T)
            out = out.detach().cpu().numpy() if hasattr(out, "detach") else np.asarray(out)
            vals.append(np.broadcast_to(out, (grid.shape[0],)) if np.ndim(out) == 0 else out)
        return np.reshape(np.concatenate([np.reshape(v, (-1,)) for v in vals]), (-1, 1))


class dirichletBC(BC):
    kind = "dirichlet"
    isDirichlect = True

    def __init__(self, domain, val, var, target):
        if target not in ("upper", "lower"):
            raise ValueError("target must be 'upper' or 'lower'")
        self.domain, self.val, self.var, self.target_name = domain, val, var, target
        self.target = domain.get_dict(var)[var + target]
        self.input = self._face_mesh(var, self.target)


class FunctionDirichletBC(BC):
    kind = "dirichlet"
    isDirichlect = True

    def __init__(self, domain, fun, var, target, func_inputs, n_values=None, replace=True):
        self.domain, self.fun, self.var, self.target_name = domain, list(fun), var, target
        self.func_inputs, self.n_values = func_inputs, n_values
        self.targets = domain.get_dict(var)[var + target]
        mesh = self._face_mesh(var, self.targets)
        self.nums = _subset(len(mesh), n_values, replace)
        self.input = mesh if self.nums is None else mesh[self.nums]
        val = self._eval_funs(self.fun, func_inputs)
        self.val = val if self.nums is None else val[self.nums]


class IC(BC):
    kind = "ic"
    isInit = True

    def __init__(self, domain, fun, var, n_values=None, replace=True, t0=None):
        if domain.time_var is None:
            raise ValueError("IC needs a domain declared with time_var")
        self.domain, self.fun, self.vars, self.n_values = domain, list(fun), var, n_values
        tv = domain.time_var
        self.t0 = domain.get_dict(tv)["range"][0] if t0 is None else float(t0)
        others = [v for v in domain.vars if v != tv]
        mesh = flatten_and_stack(multimesh([domain.linspace(v) for v in others]))
        mesh = np.insert(mesh, domain.vars.index(tv), np.full(mesh.shape[0], self.t0), axis=1)
        self.nums = _subset(len(mesh), n_values, replace)
        self.input = mesh if self.nums is None else mesh[self.nums]
        val = self._eval_funs(self.fun, var)
        self.val = val if self.nums is None else val[self.nums]


class _DerivBC(BC):
    """Shared machinery for conditions evaluated through user ``deriv_model`` callables."""

    def u_x_model(self, u_model, inputs):
        cols = inputs if isinstance(inputs, (list, tuple)) else [inputs[:, i:i + 1] for i in range(inputs.shape[1])]
        return [model(u_model, *cols) for model in self.deriv_model]

    def unroll(self, pts):
        """Reference layout: per var a ``(ndim, n, 1)`` array of columns."""
        return [np.asarray([p[:, j:j + 1] for j in range(p.shape[1])]) for p in pts]


class FunctionNeumannBC(_DerivBC):
    kind = "neumann"
    isNeumann = True

    def __init__(self, domain, fun, var, target, deriv_model, func_inputs, n_values=None,
                 replace=True):
        self.domain, self.fun, self.target_name = domain, list(fun), target
        self.var = [var] if isinstance(var, str) else list(var)
        self.deriv_model = list(deriv_model)
        self.func_inputs, self.n_values = func_inputs, n_values
        faces = [self._face_mesh(v, domain.get_dict(v)[v + target]) for v in self.var]
        self.nums = _subset(len(faces[0]), n_values, replace, force=True)
        self.points = [f[self.nums] for f in faces]
        self.input = self.unroll(self.points)
        self.val = self._eval_funs(self.fun, func_inputs)[self.nums]


class periodicBC(_DerivBC):
    kind = "periodic"
    isPeriodic = True

    def __init__(self, domain, var, deriv_model, n_values=None, replace=True):
        self.domain, self.n_values = domain, n_values
        self.var = [var] if isinstance(var, str) else list(var)
        self.deriv_model = list(deriv_model)
        up, lo = [], []
        for v in self.var:
            lo_v, hi_v = domain.get_dict(v)["range"]
            up.append(self._face_mesh(v, hi_v))
            lo.append(self._face_mesh(v, lo_v))
        self.nums = _subset(len(up[0]), n_values, replace, force=True)
        self.upper_points = [u[self.nums] for u in up]
        self.lower_points = [l[self.nums] for l in lo]
        self.upper = self.unroll(self.upper_points)
        self.lower = self.unroll(self.lower_points)
