"""Fully connected tanh network with ONE contiguous fp32 parameter buffer.

Reference: tensordiffeq/networks.py:10-20 builds ``Sequential([Dense(w, tanh, glorot_normal)...,
Dense(out, linear, glorot_normal)])`` with zero biases.  Here the same architecture keeps every
weight in a single flat tensor laid out in the Keras order the reference uses for L-BFGS and
checkpoints (per layer: kernel ``(in, out)`` row-major, then bias; utils.py:7-29).  Layers are
views into that buffer, so Adam, L-BFGS, the DP all-reduce, best-model snapshots and the HIP
jet kernels all operate on one pointer (SURVEY.md §7.1 "flat parameter buffer").
"""
from __future__ import annotations

import math

import torch
from torch import nn

_TRUNC_STD_FIX = 0.87962566103423978  # std of a unit normal truncated to [-2, 2]


def glorot_normal_(t, fan_in, fan_out, generator=None):
    """Keras ``glorot_normal``: truncated normal (|x| <= 2 sigma), sigma = sqrt(2/(fi+fo))/0.8796."""
    std = math.sqrt(2.0 / (fan_in + fan_out)) / _TRUNC_STD_FIX
    with torch.no_grad():
        vals = torch.empty(t.numel(), dtype=torch.float64)
        filled = 0
        while filled < vals.numel():
            draw = torch.randn(2 * (vals.numel() - filled) + 16, dtype=torch.float64, generator=generator)
            draw = draw[draw.abs() <= 2.0][: vals.numel() - filled]
            vals[filled:filled + draw.numel()] = draw
            filled += draw.numel()
        t.copy_((vals * std).reshape(t.shape).to(t.dtype))
    return t


def layer_offsets(layer_sizes):
    """[(w_off, b_off, fan_in, fan_out)] per dense layer + total parameter count."""
    offs, off = [], 0
    for i in range(1, len(layer_sizes)):
        fi, fo = int(layer_sizes[i - 1]), int(layer_sizes[i])
        offs.append((off, off + fi * fo, fi, fo))
        off += fi * fo + fo
    return offs, off


class TanhMLP(nn.Module):
    """``[d_in, w1, ..., wL, d_out]`` tanh MLP, linear head, flat fp32 parameters."""

    activation = "tanh"

    def __init__(self, layer_sizes, device=None, dtype=torch.float32, generator=None):
        super().__init__()
        if len(layer_sizes) < 2:
            raise ValueError("layer_sizes needs at least an input and an output width")
        self.layer_sizes = [int(s) for s in layer_sizes]
        self.offsets, n = layer_offsets(self.layer_sizes)
        self.flat = nn.Parameter(torch.zeros(n, dtype=dtype))
        with torch.no_grad():
            for (wo, bo, fi, fo) in self.offsets:
                glorot_normal_(self.flat[wo:bo].view(fi, fo), fi, fo, generator=generator)
        if device is not None:
            self.to(device)

    # -- views ---------------------------------------------------------------------------
    def kernel(self, i, src=None):
        wo, bo, fi, fo = self.offsets[i]
        return (self.flat if src is None else src)[wo:bo].view(fi, fo)

    def bias(self, i, src=None):
        wo, bo, fi, fo = self.offsets[i]
        return (self.flat if src is None else src)[bo:bo + fo]

    def weights(self, src=None):
        return [(self.kernel(i, src), self.bias(i, src)) for i in range(len(self.offsets))]

    @property
    def num_params(self):
        return self.flat.numel()

    @property
    def d_in(self):
        return self.layer_sizes[0]

    @property
    def d_out(self):
        return self.layer_sizes[-1]

    # -- forward -------------------------------------------------------------------------
    def forward(self, *xs, params=None):
        x = xs[0] if len(xs) == 1 else torch.cat(xs, dim=1)
        ws = self.weights(params)
        h = x
        for i, (k, b) in enumerate(ws):
            h = torch.addmm(b, h, k)
            if i < len(ws) - 1:
                h = torch.tanh(h)
        return h

    def summary(self):
        lines = ["Layer (type)              Output Shape     Param #",
                 "=" * 52]
        for i, (wo, bo, fi, fo) in enumerate(self.offsets):
            act = "tanh" if i < len(self.offsets) - 1 else "linear"
            lines.append(f"dense_{i} (Dense, {act:6s})   (None, {fo:<6d})    {fi * fo + fo}")
        lines.append("=" * 52)
        lines.append(f"Total params: {self.num_params}")
        return "\n".join(lines)


def neural_net(layer_sizes, device=None, generator=None):
    """Reference-named constructor (networks.py:10)."""
    return TanhMLP(layer_sizes, device=device, generator=generator)


class FlatModule(nn.Module):
    """Any user ``nn.Module`` (the reference allowed replacing ``u_model`` with a custom Keras
    model, models.py:31) trained through the same flat-buffer engine: the module's parameters
    are re-materialised as views of ``self.flat`` on every call with ``torch.func.functional_call``,
    so gradients, Adam, L-BFGS, DP all-reduce and checkpoints see one contiguous vector.  Such
    networks run on the generic nested-autograd backend."""

    activation = None

    def __init__(self, module):
        super().__init__()
        self.inner = module
        names, shapes, chunks = [], [], []
        for n, p in module.named_parameters():
            names.append(n)
            shapes.append(tuple(p.shape))
            chunks.append(p.detach().reshape(-1))
            p.requires_grad_(False)
        self._names, self._shapes = names, shapes
        self._numels = [int(torch.tensor(s).prod().item()) if s else 1 for s in shapes]
        self.flat = nn.Parameter(torch.cat(chunks).clone())
        self.layer_sizes = None

    @property
    def num_params(self):
        return self.flat.numel()

    def forward(self, *xs, params=None):
        flat = self.flat if params is None else params
        pd, off = {}, 0
        for n, s, k in zip(self._names, self._shapes, self._numels):
            pd[n] = flat[off:off + k].view(s)
            off += k
        x = xs[0] if len(xs) == 1 else torch.cat(xs, dim=1)
        return torch.func.functional_call(self.inner, pd, (x,))

    def summary(self):
        return f"FlatModule({self.inner.__class__.__name__}, params={self.num_params})\n{self.inner}"
