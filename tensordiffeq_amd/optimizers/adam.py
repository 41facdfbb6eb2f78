"""Keras-formula Adam on flat device buffers.

The reference trains with ``tf.keras.optimizers.Adam(lr=0.005, beta_1=.99)`` (models.py:49-50,
333-335), i.e. TF's ``ResourceApplyAdam``::

    m <- b1 m + (1-b1) g ;  v <- b2 v + (1-b2) g^2
    lr_t = lr * sqrt(1 - b2^t) / (1 - b1^t) ;  p <- p - lr_t * m / (sqrt(v) + eps)   (eps = 1e-7)

Self-adaptive weights are trained by gradient *ascent* with a second Adam
(fit.py:136-141) - ``sign=-1`` below.

State (m, v, step count ``t``) lives on the device; ``t`` is a device scalar so a whole training
step (forward, backward, update) can be captured into one HIP graph.  On a GPU the update runs in
one fused HIP kernel for all tensors of a step (``ops.adam``); ``torch_update`` is the reference.
"""
from __future__ import annotations

import torch


class Adam:
    """Keras-compatible constructor: ``Adam(learning_rate=0.001, beta_1=0.9, beta_2=0.999,
    epsilon=1e-7)`` (``lr=`` accepted as the legacy alias)."""

    def __init__(self, learning_rate=0.001, beta_1=0.9, beta_2=0.999, epsilon=1e-7, lr=None,
                 name="Adam", **_ignored):
        self.learning_rate = float(lr if lr is not None else learning_rate)
        self.beta_1 = float(beta_1)
        self.beta_2 = float(beta_2)
        self.epsilon = float(epsilon)
        self.name = name
        self._state = {}  # id(param) -> (m, v)
        self._t = None   # device step counter (float64)

    # -- keras-style API -----------------------------------------------------------------
    @property
    def lr(self):
        return self.learning_rate

    @lr.setter
    def lr(self, v):
        self.learning_rate = float(v)

    @property
    def iterations(self):
        return 0 if self._t is None else int(self._t.item())

    def state_for(self, p):
        st = self._state.get(id(p))
        # keyed by id(): a freed tensor's id can be reused by a new one of another shape/device
        if st is None or st[0].shape != p.shape or st[0].device != p.device:
            st = (torch.zeros_like(p), torch.zeros_like(p))
            self._state[id(p)] = st
        return st

    def step_counter(self, device):
        if self._t is None or self._t.device != torch.device(device):
            self._t = torch.zeros((), dtype=torch.float64, device=device)
        return self._t

    def apply_gradients(self, grads_and_vars, sign=1.0):
        """Keras signature: list of (grad, variable) pairs (variables updated in place)."""
        pairs = [(g, v) for g, v in grads_and_vars if g is not None]
        if not pairs:
            return
        t = self.step_counter(pairs[0][1].device)
        t.add_(1.0)
        with torch.no_grad():
            for g, v in pairs:
                m, s = self.state_for(v)
                torch_update(v, g, m, s, t, self.learning_rate, self.beta_1, self.beta_2,
                             self.epsilon, sign)

    def state_dict(self):
        return {"t": None if self._t is None else self._t.detach().cpu(),
                "hyper": (self.learning_rate, self.beta_1, self.beta_2, self.epsilon)}

    def get_config(self):
        return {"name": self.name, "learning_rate": self.learning_rate, "beta_1": self.beta_1,
                "beta_2": self.beta_2, "epsilon": self.epsilon}


def bias_corrected_lr(t, lr, b1, b2):
    """Device scalar lr * sqrt(1-b2^t)/(1-b1^t) (t is a float64 device tensor)."""
    return lr * torch.sqrt(1.0 - torch.pow(b2, t)) / (1.0 - torch.pow(b1, t))


def torch_update(p, g, m, v, t, lr, b1, b2, eps, sign=1.0):
    """Reference Keras Adam step (in place).  ``t`` already incremented."""
    g = g if sign == 1.0 else g * sign
    m.mul_(b1).add_(g, alpha=1.0 - b1)
    v.mul_(b2).addcmul_(g, g, value=1.0 - b2)
    lr_t = bias_corrected_lr(t, lr, b1, b2).to(p.dtype)
    p.sub_(lr_t * m / (v.sqrt() + eps))
