"""N-D box domains (reference tensordiffeq/domains.py:1-31).

``DomainND(var, time_var)`` declares the axes; ``add(token, vals, fidel)`` stores a per-axis dict
with the same keys as the reference (``identifier``, ``range``, ``<v>fidelity``, ``<v>linspace``,
``<v>upper``, ``<v>lower``) so user code indexing ``domain.domaindict[0]['xlinspace']`` keeps
working.  ``generate_collocation_points`` builds ``X_f`` (N_f x ndim, float64, host) with the
package LHS sampler; ``device=...`` builds it directly on a GPU instead (large N_f).
"""
from __future__ import annotations

import numpy as np

from .sampling import LatinHypercubeSample, lhs_device


class DomainND:
    def __init__(self, var, time_var=None):
        self.vars = list(var)
        self.domaindict = []
        self.domain_ids = []
        self.time_var = time_var
        self.X_f = None

    def add(self, token, vals, fidel):
        if token not in self.vars:
            raise ValueError(f"variable {token!r} is not one of the domain variables {self.vars}")
        lo, hi = float(vals[0]), float(vals[1])
        self.domain_ids.append(token)
        self.domaindict.append({
            "identifier": token,
            "range": [lo, hi],
            token + "fidelity": int(fidel),
            token + "linspace": np.linspace(lo, hi, int(fidel)),
            token + "upper": hi,
            token + "lower": lo,
        })

    # -- queries -------------------------------------------------------------------------
    def get_dict(self, var):
        return next(d for d in self.domaindict if d["identifier"] == var)

    def linspace(self, var):
        return self.get_dict(var)[var + "linspace"]

    def bounds(self):
        """``(ndim, 2)`` array of [lower, upper] in ``self.vars`` order."""
        return np.array([self.get_dict(v)["range"] for v in self.vars], dtype=np.float64)

    @property
    def ndim(self):
        return len(self.vars)

    def generate_collocation_points(self, N_f, criterion="c", random_state=None, device=None,
                                    generator=None):
        missing = [v for v in self.vars if v not in self.domain_ids]
        if missing:
            raise ValueError(f"domain variables {missing} were never added")
        limits = self.bounds()
        if device is not None:
            self.X_f = lhs_device(int(N_f), limits, device, generator=generator)
        else:
            self.X_f = LatinHypercubeSample(int(N_f), limits, criterion=criterion,
                                            random_state=random_state)
        return self.X_f
