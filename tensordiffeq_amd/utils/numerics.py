"""Loss primitives, dtype helpers and flat-parameter helpers.

Parity map (reference tensordiffeq/utils.py):
  MSE                      utils.py:38-44   mean((w*(p-a))^2) | w*mean((p-a)^2) | mean((p-a)^2)
  g_MSE                    utils.py:47-48   mean(g(lam)*(p-a)^2)
  constant/convertTensor/tensor  utils.py:51-69
  get_sizes                utils.py:32-35
  get_weights/set_weights  utils.py:7-29    flat vector <-> per-layer (kernel(in,out) row-major, bias)
  initialize_weights_loss  utils.py:102-115 builds the SA lambda list + index map

Differences by design: tensors are torch tensors; ``get_weights``/``set_weights`` operate on the
flat parameter buffer of :class:`tensordiffeq_amd.models.networks.TanhMLP` (no host round trip),
and fall back to per-layer copies for arbitrary ``nn.Module`` networks.
"""
from __future__ import annotations

import torch

DEFAULT_DTYPE = torch.float32


def _sq(x):
    return x * x


def MSE(pred, actual, weights=None, outside_sum=False, denom=None):
    """Mean squared error with optional self-adaptive weights.

    ``denom`` overrides the mean's denominator (used by data-parallel sharding so that the
    per-rank partial sums add up to the global mean).
    """
    diff = pred - actual
    if weights is not None:
        if outside_sum:
            return (weights * _mean(_sq(diff), denom)).sum()
        return _mean(_sq(weights * diff), denom)
    return _mean(_sq(diff), denom)


def g_MSE(pred, actual, g_lam, denom=None):
    return _mean(g_lam * _sq(pred - actual), denom)


def _mean(x, denom):
    if denom is None:
        return x.mean()
    return x.sum() / denom


def constant(val, dtype=DEFAULT_DTYPE):
    return torch.tensor(val, dtype=dtype)


def convertTensor(val, dtype=DEFAULT_DTYPE, device=None):
    if isinstance(val, torch.Tensor):
        return val.to(dtype=dtype, device=device if device is not None else val.device)
    return torch.as_tensor(val, dtype=dtype, device=device)


def tensor(x, dtype=DEFAULT_DTYPE, device=None):
    return convertTensor(x, dtype=dtype, device=device)


def get_tf_model(model):
    """Reference wraps user callables in ``tf.function``; eager torch needs no wrapping."""
    return model


get_model = get_tf_model


def get_sizes(layer_sizes):
    sizes_w = [layer_sizes[i] * layer_sizes[i - 1] for i in range(1, len(layer_sizes))]
    sizes_b = list(layer_sizes[1:])
    return sizes_w, sizes_b


def get_weights(model):
    """Flat parameter vector in Keras order (per layer: kernel(in,out) row-major, then bias)."""
    flat = getattr(model, "flat", None)
    if flat is not None:
        return flat.detach().clone()
    parts = []
    for layer in _linear_layers(model):
        parts.append(layer.weight.detach().t().reshape(-1))
        parts.append(layer.bias.detach().reshape(-1))
    return torch.cat(parts)


def set_weights(model, w, sizes_w=None, sizes_b=None):
    flat = getattr(model, "flat", None)
    with torch.no_grad():
        if flat is not None:
            flat.copy_(torch.as_tensor(w, dtype=flat.dtype, device=flat.device).reshape(-1))
            return
        off = 0
        for layer in _linear_layers(model):
            n_in, n_out = layer.in_features, layer.out_features
            k = torch.as_tensor(w[off:off + n_in * n_out]).reshape(n_in, n_out)
            layer.weight.copy_(k.t())
            off += n_in * n_out
            layer.bias.copy_(torch.as_tensor(w[off:off + n_out]))
            off += n_out


def _linear_layers(model):
    return [m for m in model.modules() if isinstance(m, torch.nn.Linear)]


def initialize_weights_loss(init_weights, adaptive_map, device=None):
    """Create trainable SA weights for every term marked adaptive with a non-None initial value.

    Returns ``(lambdas, lambdas_map)`` where ``lambdas_map[key.lower()]`` lists indices into
    ``lambdas`` in term order (reference utils.py:102-115).
    """
    lambdas, lambdas_map, counter = [], {}, 0
    for key, values in init_weights.items():
        idx = []
        for j, value in enumerate(values):
            if value is not None and adaptive_map[key][j] is not False:
                t = torch.as_tensor(value, dtype=DEFAULT_DTYPE)
                if device is not None:
                    t = t.to(device)
                lambdas.append(t.detach().clone().reshape(-1, 1) if t.dim() > 0 else t.detach().clone())
                idx.append(counter)
                counter += 1
        lambdas_map[key.lower()] = idx
    return lambdas, lambdas_map
