"""Latin-hypercube sampling of collocation points.

Behaviour (reference tensordiffeq/sampling.py:257-313, a vendored SMT ``LHS``): points are drawn
on the unit cube and scaled to ``xlimits``; the default criterion ``'c'`` places every point at
the centre of its stratum with an independent random permutation per dimension (B21).

This is an independent implementation.  Criteria:
  ``'c'/'center'``             stratum centres, permuted per dim (default)
  ``'r'/'random'``             uniform jitter inside each stratum
  ``'m'/'maximin'``            best of ``iterations`` jittered designs by max-min distance
  ``'cm'/'centermaximin'``     best of ``iterations`` centred designs by max-min distance
  ``'corr'/'correlation'``     best of ``iterations`` designs by min max |corr|
  ``'ese'``                    enhanced stochastic evolutionary optimisation of the phi_p criterion

``lhs_device`` builds the centred design directly on the GPU (used for multi-million point
domains where the host build and H2D copy would dominate set-up time).
"""
from __future__ import annotations

import numpy as np
import torch

_ALIASES = {
    "c": "center", "center": "center",
    "r": "random", "random": "random",
    "m": "maximin", "maximin": "maximin",
    "cm": "centermaximin", "centermaximin": "centermaximin",
    "corr": "correlation", "correlation": "correlation",
    "ese": "ese",
}


def _rng(random_state):
    if isinstance(random_state, np.random.RandomState):
        return random_state
    if isinstance(random_state, np.random.Generator):
        return np.random.RandomState(int(random_state.integers(0, 2**31 - 1)))
    if random_state is None:
        from .utils import seeding
        return seeding.numpy_rng()
    return np.random.RandomState(int(random_state))


def _unit_lhs(n, d, rng, centered):
    u = np.empty((n, d))
    for j in range(d):
        perm = rng.permutation(n)
        off = 0.5 if centered else rng.uniform(size=n)
        u[:, j] = (perm + off) / n
    return u


def _min_dist(x):
    if len(x) < 2:
        return np.inf
    sq = np.sum(x * x, axis=1)
    d2 = sq[:, None] + sq[None, :] - 2.0 * x @ x.T
    np.fill_diagonal(d2, np.inf)
    return float(np.sqrt(max(d2.min(), 0.0)))


def _max_abs_corr(x):
    if x.shape[1] < 2:
        return 0.0
    c = np.corrcoef(x, rowvar=False)
    np.fill_diagonal(c, 0.0)
    return float(np.max(np.abs(c)))


def _phi_p(x, p=10.0):
    diff = x[:, None, :] - x[None, :, :]
    d = np.sqrt(np.sum(diff * diff, axis=-1))
    iu = np.triu_indices(len(x), 1)
    dd = np.maximum(d[iu], 1e-300)
    return float(np.sum(dd ** (-p)) ** (1.0 / p))


def _ese(x, rng, outer=None, inner=None, p=10.0):
    """Enhanced stochastic evolutionary algorithm (Jin, Chen & Sudjianto 2005) on phi_p.

    Each inner step tries ``J`` random pair exchanges inside one column and keeps the best;
    the acceptance threshold adapts on the outer loop.
    """
    n, d = x.shape
    if n < 3:
        return x
    outer = outer or min(int(1.5 * d), 30) or 1
    inner = inner or min(20 * d, 100)
    J = min(max(n // 5, 1), 50)
    x_best = x.copy()
    phi = phi_best = _phi_p(x, p)
    thresh = 0.005 * phi
    for _ in range(outer):
        n_acc = n_imp = 0
        for it in range(inner):
            col = it % d
            best_try, best_phi = None, np.inf
            for _ in range(J):
                a, b = rng.choice(n, 2, replace=False)
                y = x.copy()
                y[[a, b], col] = y[[b, a], col]
                ph = _phi_p(y, p)
                if ph < best_phi:
                    best_try, best_phi = y, ph
            if best_phi - phi <= thresh * rng.uniform():
                x, phi = best_try, best_phi
                n_acc += 1
                if phi < phi_best:
                    x_best, phi_best = x.copy(), phi
                    n_imp += 1
        ratio = n_acc / inner
        if n_imp > 0:
            thresh *= 0.8 if ratio > 0.1 else 1.0
        else:
            thresh *= 1.25 if ratio < 0.8 else 0.9
    return x_best


def lhs_unit(n, d, criterion="c", random_state=None, iterations=5):
    crit = _ALIASES.get(criterion)
    if crit is None:
        raise ValueError(f"unknown LHS criterion {criterion!r}")
    rng = _rng(random_state)
    if crit in ("center", "random"):
        return _unit_lhs(n, d, rng, centered=(crit == "center"))
    if crit in ("maximin", "centermaximin"):
        centered = crit == "centermaximin"
        best, best_score = None, -np.inf
        for _ in range(max(1, iterations)):
            cand = _unit_lhs(n, d, rng, centered)
            score = _min_dist(cand) if n <= 4000 else _min_dist(cand[rng.choice(n, 4000, replace=False)])
            if score > best_score:
                best, best_score = cand, score
        return best
    if crit == "correlation":
        best, best_score = None, np.inf
        for _ in range(max(1, iterations)):
            cand = _unit_lhs(n, d, rng, False)
            score = _max_abs_corr(cand)
            if score < best_score:
                best, best_score = cand, score
        return best
    # ese
    return _ese(_unit_lhs(n, d, rng, centered=True), rng)


def scale_to_limits(u, xlimits):
    xlimits = np.asarray(xlimits, dtype=np.float64)
    return xlimits[:, 0] + u * (xlimits[:, 1] - xlimits[:, 0])


class OptionsDictionary(dict):
    """Declared options with defaults / allowed values / types (the SMT options object the
    reference's sampler carries, ``sampling.py:14-146``)."""

    def __init__(self):
        super().__init__()
        self._decl = {}

    def declare(self, name, default=None, values=None, types=None, desc=""):
        self._decl[name] = {"default": default, "values": values, "types": types, "desc": desc}
        if name not in self:
            dict.__setitem__(self, name, default)

    def __setitem__(self, name, value):
        d = self._decl.get(name)
        if d is None:
            raise KeyError(f"option {name!r} was not declared")
        if d["values"] is not None and value not in d["values"]:
            raise ValueError(f"option {name!r}: {value!r} not in {d['values']}")
        if d["types"] is not None and value is not None and not isinstance(value, d["types"]):
            raise TypeError(f"option {name!r}: {type(value).__name__} is not {d['types']}")
        dict.__setitem__(self, name, value)

    def update(self, other=(), **kw):
        for k, v in dict(other, **kw).items():
            self[k] = v


class SamplingMethod:
    """Base sampler: ``sampler(nt) -> (nt, nx)`` points (reference ``sampling.py:148-198``)."""

    def __init__(self, **kwargs):
        self.options = OptionsDictionary()
        self.options.declare("xlimits", types=np.ndarray, desc="(nx, 2) bounds per dimension")
        self._initialize()
        if "xlimits" in kwargs:
            kwargs["xlimits"] = np.asarray(kwargs["xlimits"], dtype=np.float64)
        self.options.update(kwargs)

    def _initialize(self):
        pass

    def __call__(self, nt):
        return self._compute(int(nt))

    def _compute(self, nt):
        raise NotImplementedError


class ScaledSamplingMethod(SamplingMethod):
    """Samples on the unit hypercube, then maps to ``xlimits`` (reference ``sampling.py:201-254``)."""

    def __call__(self, nt):
        return scale_to_limits(self._compute(int(nt)), self.options["xlimits"])


class LHS(ScaledSamplingMethod):
    """Latin hypercube: ``LHS(xlimits=..., criterion='c', random_state=None)`` (reference
    ``sampling.py:257-313``); criteria c/center, m/maximin, cm/centermaximin, corr/correlation, ese."""

    def __init__(self, xlimits=None, criterion="c", random_state=None, iterations=5, **kw):
        super().__init__(xlimits=xlimits, criterion=criterion, random_state=random_state, iterations=iterations,
                         **kw)

    def _initialize(self):
        o = self.options
        o.declare("criterion", "c", values=["center", "maximin", "centermaximin", "correlation", "c", "m", "cm",
                                            "corr", "ese"])
        o.declare("random_state", None)
        o.declare("iterations", 5, types=int)

    def _compute(self, nt):
        o = self.options
        return lhs_unit(nt, o["xlimits"].shape[0], o["criterion"], o["random_state"], o["iterations"])


def LatinHypercubeSample(N_f, bounds, criterion="c", random_state=None):
    return LHS(xlimits=bounds, criterion=criterion, random_state=random_state)(N_f)


def lhs_device(n, xlimits, device, generator=None, dtype=torch.float32):
    """Centred LHS generated on ``device`` (one ``randperm`` per dimension)."""
    xl = torch.as_tensor(np.asarray(xlimits, dtype=np.float64), dtype=torch.float64, device=device)
    d = xl.shape[0]
    cols = []
    for _ in range(d):
        perm = torch.randperm(n, device=device, generator=generator, dtype=torch.int64)
        cols.append((perm.to(torch.float64) + 0.5) / n)
    u = torch.stack(cols, dim=1)
    return (xl[:, 0] + u * (xl[:, 1] - xl[:, 0])).to(dtype)
