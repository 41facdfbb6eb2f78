"""Loader for the in-tree native library ``libtdq_hip.so`` (HIP kernels for gfx950).

The kernels are plain HIP C++ compiled by ``hipcc --offload-arch=gfx950`` (see
``tensordiffeq_amd/csrc/build.py``) and exported through a small C ABI; Python passes device
pointers and the current HIP stream (``torch.cuda.current_stream().cuda_stream``), so launches
are captured by torch's HIP-graph capture like any other kernel on that stream.

Policy: on a machine with a GPU, a missing or stale library is an ERROR (never a silent torch
fallback) unless ``TDQ_ALLOW_TORCH_FALLBACK=1`` is set; on CPU-only machines the torch
implementations are used.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TDQ_LIB_PATH") or os.path.join(os.path.dirname(_HERE), "csrc", "libtdq_hip.so")
ABI_VERSION = 27

_lock = threading.Lock()
_lib = None
_err = None


class NativeUnavailable(RuntimeError):
    pass


def _declare(lib):
    c = ctypes
    P, I, F, L, D = c.c_void_p, c.c_int, c.c_float, c.c_int64, c.c_double
    sig = {
        "tdq_abi_version": (I, []),
        "tdq_jet_fwd": (I, [P, P, P, P, I, I, I, I, I, I, P, P]),
        "tdq_jet_bwd": (I, [P, P, P, P, P, P, I, I, I, I, I, I, P, P]),
        "tdq_jet_scratch_floats": (L, [I, I, I, I, I]),
        "tdq_jet_slab_floats": (L, [I, I, I, I, I]),
        # split-bf16 family: `widths` = pointer to the n_hidden hidden-layer widths
        "tdq_jet_fwd_bf3": (I, [P, P, P, P, I, I, P, I, I, I, P, I, P]),
        "tdq_jet_bwd_bf3": (I, [P, P, P, P, P, P, I, I, P, I, I, I, P, I, P]),
        "tdq_jet_fwd_bf3_ex": (I, [P, P, P, P, I, I, P, I, I, I, P, I, I, P]),
        "tdq_jet_bwd_bf3_ex": (I, [P, P, P, P, P, P, I, I, P, I, I, I, P, I, I, P]),
        "tdq_jet_fwd_bf3_range": (I, [P, P, P, P, I, I, I, I, P, I, I, I, P, I, I, P]),
        "tdq_jet_bwd_bf3_range": (I, [P, P, P, P, I, I, I, I, P, I, I, I, P, I, P]),
        "tdq_jet_bf3_pack": (I, [P, P, I, I, P, I, I, I, P]),
        "tdq_step_tail_bf3": (I, [P, P, P, I, I, P, I, I, I, I, P, I, I, I, P, P, P] + [P, L, P, P, P, P]
                              + [P, I, P, I, P, I, P, I, P]),
        "tdq_bf3_slab_geometry": (I, [I, I, P, I, I, I, I, P]),
        "tdq_slab_prereduce_bf3": (I, [P, I, I, P, I, I, I, I, I, I, P]),
        "tdq_dp_tail_a_bf3": (I, [P, P, I, I, P, I, I, I, I, P, I, I, I, P, P, P, I, P, I, I, P]),
        "tdq_dp_tail_b_bf3": (I, [P, I, I, P, I, I, I, P, I, P, P, P]),
        "tdq_jet_bf3_scratch_floats": (L, [I, I, P, I, I, I]),
        "tdq_jet_bf3_slab_floats": (L, [I, I, P, I, I]),
        # persistent point-tile kernels (csrc/jet_fused.h) behind the split-bf16 entry points
        "tdq_fused_step_launch": (I, [P, P, P, P, I, I, P, I, I, I, P, I, I, I, P, P, I, I, I, P]),
        "tdq_fused_params_size": (I, []),
        "tdq_jet_fused_lds": (I, [I, P, I, I, I, I]),
        "tdq_device_cus": (I, []),
        "tdq_slab_floats_rows": (L, [I, I, P, I, I]),
        # hand-written GEMMs of the layer-wise engine (csrc/lay_gemm.hip, ops/jet_layered.py)
        "tdq_lay_nn": (I, [I, P, P, L, P, P, L, P, L, I, I, I, P]),
        "tdq_lay_tn": (I, [I, P, P, L, P, P, L, P, I, I, I, I, P]),
        "tdq_lay_xtz": (I, [P, I, P, I, I, P, I, P]),
        "tdq_lay_xtz2": (I, [P, I, P, P, P, I, I, P, I, P]),
        "tdq_colsum_work": (L, [I, L]),
        "tdq_colsum": (I, [P, L, I, L, P, L, L, L, P, L, I, P, P]),
        "tdq_lay_bplanes": (I, [P, I, I, I, P, P, P]),
        "tdq_lay_l0grad": (I, [P, I, I, P, I, P, P, P]),
        "tdq_lay_nnj": (I, [I, I, I, P, P, P, P, P, I, I, I, P, P, P, P, P, P, P, I, P, P, I, P]),
        "tdq_lay_in_fwd": (I, [I, I, P, P, I, P, P, I, I, P, P, P]),
        "tdq_lay_out_bwd": (I, [I, I, I, P, P, I, P, P, P, I, I, P, P, P, P, I, P]),
        "tdq_adam_multi": (I, [P, I, P, P, P]),
        "tdq_step_book": (I, [P, P, I, I, P, L, P, P, P, P, P, I, P]),
        "tdq_best_track": (I, [P, P, P, P, P, P, L, P]),
        "tdq_loss_fused": (I, [P, P, P, P, P, I, I, I, I, I, I, P, P, P, P, I, I, P, P, P, I, I, P]),
        "tdq_loss_fused_range": (I, [P, P, P, P, P, I, I, I, I, I, I, P, P, P, P, I, I, I, I, P]),
        "tdq_loss_meta_sizes": (I, [P]),
        "tdq_loss_reduce_partials": (I, [P, I, I, I, P, P, P, I, P]),
        "tdq_lbfgs_nst": (I, []),
        "tdq_lbfgs_ticket_ints": (I, []),
        "tdq_lbfgs_update": (I, [P] * 14 + [I] * 6 + [D] * 4 + [I, P]),
        "tdq_lbfgs_axpy": (I, [P, P, P, I, I, P]),
        "tdq_lbfgs_update_fused": (I, [P] * 16 + [I] * 6 + [D] * 4 + [I, P, P]),
        "tdq_img_target": (I, [P, I, P, I, I, P, I]),
        "tdq_layered_epi": (I, [I, P, P, P, L, I, I, P, P, P, P, P, P]),
        # high-order (<= 4) jets of small point sets (csrc/jet_hi.hip, ops/jet_hi.py)
        "tdq_jet_hi_scratch_floats": (L, [I, I]),
        "tdq_jet_hi_work_floats": (L, [I, I, P, I, I]),
        "tdq_jet_hi_fwd": (I, [P, I, P, I, P, I, I, P, P, P, I, I, P, P]),
        "tdq_jet_hi_bwd": (I, [P, I, P, I, P, I, I, P, P, P, I, I, P, P, P, P]),
        "tdq_jet_hi_bwd_part": (I, [P, I, P, I, P, I, I, P, P, P, I, I, P, P, P, I, P]),
        "tdq_jet_hi_limits": (I, [P]),
        "tdq_jet_hi_lds_ok": (I, [I, I, I, I]),
        # one-shot peer-memory all-reduce (csrc/peer.hip, parallel/peer.py)
        "tdq_peer_maxw": (I, []),
        "tdq_peer_chunk": (I, []),
        "tdq_peer_alloc": (I, [L, I, P]),
        "tdq_peer_free": (I, [P]),
        "tdq_peer_ipc_handle": (I, [P, P]),
        "tdq_peer_ipc_open": (I, [P, P]),
        "tdq_peer_ipc_close": (I, [P]),
        "tdq_peer_allreduce": (I, [P, I, I, I, L, I, P, P, P, P, L, P]),
        # run-time specialized fused-loss kernels (csrc/loss_jit.hip, ops/loss_jit.py)
        "tdq_rtc_compile": (I, [c.c_char_p, c.c_char_p, c.c_char_p, P, P, c.c_char_p, I]),
        "tdq_rtc_compile_ex": (I, [c.c_char_p, c.c_char_p, c.c_char_p, c.c_char_p, P, P, c.c_char_p, I]),
        "tdq_rtc_free": (None, [P]),
        "tdq_rtc_load": (I, [P, c.c_char_p, P, P]),
        "tdq_rtc_unload": (I, [P]),
        "tdq_rtc_set_global_ptr": (I, [P, c.c_char_p, P]),
        "tdq_loss_jit_range": (I, [P, P, P, P, P, P, I, I, P]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.restype = res
        fn.argtypes = args


def load(required=None):
    """Return the ctypes library or raise :class:`NativeUnavailable`."""
    global _lib, _err
    with _lock:
        if _lib is not None:
            return _lib
        if _err is not None and not required:
            raise NativeUnavailable(_err)
        if not os.path.exists(LIB_PATH):
            _err = f"{LIB_PATH} not built (run `python -m tensordiffeq_amd.csrc.build`)"
            raise NativeUnavailable(_err)
        try:
            lib = ctypes.CDLL(LIB_PATH)
            _declare(lib)
            ver = lib.tdq_abi_version()
            if ver != ABI_VERSION:
                _err = f"libtdq_hip.so ABI {ver} != expected {ABI_VERSION}; rebuild"
                raise NativeUnavailable(_err)
            built, want = library_hash(lib), expected_hash()
            if want is not None and built != want and os.environ.get("TDQ_SKIP_HASH_CHECK", "0") != "1":
                _err = (f"{LIB_PATH} is stale: built from sources {built}, the csrc/ sources hash to {want} "
                        f"(run `python -m tensordiffeq_amd.csrc.build`)")
                raise NativeUnavailable(_err)
        except OSError as e:
            _err = f"cannot load {LIB_PATH}: {e}"
            raise NativeUnavailable(_err)
        _lib = lib
        return _lib


def library_hash(lib):
    """Source hash the library was built from (``tdq_src_hash``), or None for an old build."""
    fn = getattr(lib, "tdq_src_hash", None)
    if fn is None:
        return None
    fn.restype = ctypes.c_char_p
    fn.argtypes = []
    return fn().decode()


def expected_hash():
    """Hash of the HIP sources next to the library (None when they are not shipped)."""
    from ..csrc import build as _build
    if not _build.source_files():
        return None
    return _build.source_hash()


def available():
    try:
        load()
        return True
    except NativeUnavailable:
        return False


def fallback_allowed():
    return os.environ.get("TDQ_ALLOW_TORCH_FALLBACK", "0") == "1"


def gpu_present():
    try:
        return torch.cuda.is_available()
    except Exception:  # pragma: no cover
        return False


def require_on_gpu():
    """Raise when running on a GPU without the native library (unless fallback is allowed)."""
    if gpu_present() and not fallback_allowed():
        load(required=True)


def stream_ptr(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed with HIP error {rc}")


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)
