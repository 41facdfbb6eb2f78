"""Jet evaluation of a tanh MLP: dispatch between the torch engine and the fused HIP kernels.

``jet_eval(X, net, params, plan, backend)`` returns ``J`` of shape ``(S, N, d_out)`` (stream-major,
streams in ``plan.streams`` order) and is differentiable w.r.t. ``params`` (the flat buffer).

HIP path (``backend="hip"``, MI355X): two kernels from ``csrc/jet_mlp.hip``

* ``tdq_jet_fwd``  one workgroup = 4 waves x 16 points.  The whole layer stack runs on chip:
  activations for all derivative streams stay in VGPRs in a *feature-major* MFMA layout
  (point on the lane, features in registers), so each layer's output accumulator is directly
  the next layer's B operand - no LDS round trip between layers.  Hidden GEMMs use
  ``v_mfma_f32_16x16x4_f32`` (exact fp32) with the layer's weights staged in LDS; the tanh-jet
  epilogue (Faa di Bruno, order <= 2) is fused.  Pre-activations of every hidden layer are
  written in register-image order (256-B coalesced) for the backward.
* ``tdq_jet_bwd``  reverse pass through the same stack: recomputes tanh / its derivatives from the
  saved pre-activations, chains the stream adjoints through ``W^T`` on MFMA, and accumulates
  ``dW = sum_points sum_streams zbar h^T`` per workgroup through an LDS transpose into MFMA,
  writing one partial slab per workgroup; a deterministic reduction kernel folds the slabs into
  the flat gradient (Keras order).
"""
from __future__ import annotations

import os

import torch

from ..jet import jet_forward
from . import _lib

MAX_S = 8
PTS_PER_WG = 64
PRECISIONS = ("bf16x3", "bf16", "fp32")
_precision = os.environ.get("TDQ_PRECISION", "bf16x3")


def set_precision(p):
    """Default GEMM precision of the HIP jet kernels: ``"bf16x3"`` (split-bf16 MFMA, ~2^-16 relative
    error per product, default), ``"bf16"`` (weights and activations rounded to bf16, one MFMA
    per product, fp32 accumulation; two workgroups per CU) or
    ``"fp32"`` (exact-fp32 MFMA)."""
    global _precision
    if p not in PRECISIONS:
        raise ValueError(f"precision must be one of {PRECISIONS}")
    _precision = p


def get_precision():
    return _precision


def _pad16(w):
    return (w + 15) // 16 * 16


def hip_config(net, plan, precision=None):
    """Return the kernel geometry or raise ValueError if the kernels cannot serve it.

    ``precision`` (default: :func:`get_precision`) picks the kernel family; bf16x3 needs at least
    two 16-feature tiles (width > 16) and falls back to fp32 below that (so does bf16)."""
    sizes = net.layer_sizes
    d_in, d_out = sizes[0], sizes[-1]
    hidden = sizes[1:-1]
    if len(hidden) < 1:
        raise ValueError("needs at least one hidden layer")
    if plan.order > 2:
        raise ValueError("derivative order > 2")
    S = plan.S
    if S > MAX_S:
        raise ValueError(f"{S} streams > {MAX_S}")
    uniform = len(set(hidden)) == 1
    wpad = _pad16(max(hidden))
    WT = wpad // 16
    precision = precision or _precision
    if precision not in PRECISIONS:
        raise ValueError(f"precision {precision!r} not in {PRECISIONS}")

    def layered(why):
        # outside the fused kernels' envelope: the layer-wise engine (library GEMMs on the stacked
        # streams in the requested precision family + fused HIP tanh-jet epilogues,
        # ops/jet_layered.py), which takes any depth, width and input / output width
        return {"d_in": d_in, "d_out": d_out, "width": max(hidden), "widths": tuple(hidden), "WT": WT, "S": S,
                "n_hidden": len(hidden), "precision": precision, "engine": "layered", "why": why}

    if WT > 16:
        return layered("hidden width > 256")
    if WT > 8:
        # widths 129..256: the split-bf16 kernels at WT = 16 in bf16 with S <= 4 (csrc/jet_bf3_w16.hip);
        # fp32 / bf16x3 there keep the layer-wise engine
        if precision != "bf16":
            return layered(f"hidden width > 128 in {precision}")
        if S > 4:
            return layered("hidden width > 128 with more than 4 streams")
        WT = 16
    if len(hidden) > 16:
        return layered("more than 16 hidden layers")
    if d_in > 8 or d_out > 4:
        return layered("input width > 8 or output width > 4")
    if WT not in (1, 2, 4, 8, 16):
        WT = 4 if WT == 3 else 8
    if precision in ("bf16x3", "bf16") and WT < 2:
        precision = "fp32"
    # split-bf16 kernels: any S <= 8 at every width class (S x WT > 32: the one-wave-per-SIMD
    # "wide" kernels, csrc/jet_bf3.h); the exact-fp32 family keeps the 2-wave register budget
    if precision == "fp32" and S * WT > 32:
        return layered(f"fp32 with streams x width tiles = {S * WT} > 32")
    if precision == "fp32" and not uniform:
        # the exact-fp32 fused family takes equal widths only; unequal widths keep the requested
        # precision on the layer-wise engine (no silent switch to split-bf16)
        return layered("unequal hidden widths in fp32")
    return {"d_in": d_in, "d_out": d_out, "width": max(hidden), "widths": tuple(hidden), "WT": WT, "S": S,
            "n_hidden": len(hidden), "precision": precision}


def hip_eligible(net, plan, device):
    from ..models.networks import TanhMLP
    if torch.device(device).type != "cuda":
        return False, "device is not a GPU"
    if not isinstance(net, TanhMLP):
        return False, "network is not a TanhMLP"
    try:
        hip_config(net, plan)
    except ValueError as e:
        return False, str(e)
    if not _lib.available():
        if _lib.fallback_allowed():
            return False, "native library unavailable (fallback allowed)"
        _lib.load(required=True)
    return True, ""


def jet_eval(X, net, params, plan, backend, precision=None):
    if backend == "jet":
        # float64 parameters: the whole jet in float64 (the fp64 oracle of smoke() / the tests)
        return jet_forward(X.to(params.dtype) if params.dtype == torch.float64 else X, net.weights(params), plan)
    if backend == "hip":
        from . import jet_hip
        return jet_hip.JetMLPFunction.apply(X, params, net, plan, precision)
    raise ValueError(f"jet_eval backend {backend!r}")
