"""Run-time specialized fused-loss kernels (hipRTC; host side ``csrc/loss_jit.hip``).

The fused loss (:mod:`.loss_fused`, ``csrc/loss_fused.hip``) interprets a traced per-point
bytecode with its SSA registers in LDS.  Once ``compile()`` has traced the user's callables the
program never changes, so :func:`generate` emits it as straight-line HIP C++ - one block of code per
segment group, registers as VGPR locals, constants as exact hex-float literals, the group table as
compile-time branches - and :class:`LossKernel` compiles it with hipRTC for the device (``gfx950``)
the first time a program with that source is built in the process.  Every statement mirrors the
interpreter's statement for the same opcode and the kernel is compiled with statement-level FMA
contraction only, with the interpreter's grid, block mapping, block reductions and output order:
the two produce the same bits (tests/test_loss_jit_gpu.py).

``TDQ_LOSS_JIT=0`` keeps the interpreter; a program the generator or hipRTC cannot handle falls
back to it with a warning.
"""
from __future__ import annotations

import ctypes
import hashlib
import math
import os
import warnings

import numpy as np

from . import _lib
from ..fusion import OP

LF_BLOCK = 128
_OPN = {v: k for k, v in OP.items()}
_CACHE = {}   # source sha -> (module, func): one compile per distinct program per process

# hipRTC provides the HIP device API implicitly (no include: under rocprofv3 the include paths of a
# run-time compile are not set up, gpurun_out r3v)
PRELUDE = r"""
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp<0xB1>(v);
  v += dpp<0x4E>(v);
  v += dpp<0x141>(v);
  v += dpp<0x140>(v);
  return v;
}
struct LFPtrs {
  const float* val[16];
  const float* lam[8];
  float* dlam[8];
  const float* scal[8];
};
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = row16_sum(v);
  const int t = threadIdx.x;
  __syncthreads();
  if ((t & 15) == 0) red[t >> 4] = v;
  __syncthreads();
  float s = 0.f;
  if (t == 0) {
#pragma unroll
    for (int k = 0; k < 128 / 16; ++k) s += red[k];
  }
  return s;
}
"""


def enabled():
    return os.environ.get("TDQ_LOSS_JIT", "1") != "0"


def _lit(x):
    """Exact float32 literal."""
    f = float(np.float32(x))
    if math.isnan(f):
        return "__builtin_nanf(\"\")"
    if math.isinf(f):
        return "__builtin_inff()" if f > 0 else "(-__builtin_inff())"
    return f"{f.hex()}f"


def _forward_code(P, e, load):
    """The program's forward statements; ``load(name, r, a, b)``: the statement of an input opcode
    (STREAM / COORD / VAL / LAM / SCAL)."""
    consts = P.consts
    for op, r, a, b in P.code:
        name = _OPN[op]
        if name in ("STREAM", "COORD", "VAL", "LAM", "SCAL"):
            e(load(name, r, a, b))
        elif name == "CONST":
            e(f"    v{r} = {_lit(consts[a])};")
        elif name in ("ADD", "SUB", "MUL", "DIV"):
            sym = {"ADD": "+", "SUB": "-", "MUL": "*", "DIV": "/"}[name]
            e(f"    v{r} = v{a} {sym} v{b};")
        elif name == "NEG":
            e(f"    v{r} = -v{a};")
        elif name == "POWI":
            e(f"    {{ const float x = v{a}; float p = 1.f;" + " p *= x;" * int(b) + f" v{r} = p; }}")
        elif name == "POWF":
            e(f"    v{r} = powf(v{a}, {_lit(consts[b])});")
        elif name in ("SIN", "COS", "EXP", "TANH", "LOG", "SQRT"):
            e(f"    v{r} = {name.lower()}f(v{a});")
        elif name == "SQUARE":
            e(f"    {{ const float x = v{a}; v{r} = x * x; }}")
        else:
            raise ValueError(f"loss JIT: opcode {op}")


def _reverse_code(P, e, store):
    """The program's reverse sweep (adjoints ``a<r>``); ``store(name, r, a, b, g)``: the statement
    of an input opcode's adjoint (STREAM / LAM / SCAL; None: nothing)."""
    consts = P.consts
    for op, r, a, b in reversed(P.code):
        name = _OPN[op]
        g = f"a{r}"
        if name in ("STREAM", "LAM", "SCAL"):
            e(store(name, r, a, b, g))
        elif name == "ADD":
            e(f"    {{ const float g = {g}; a{a} += g; a{b} += g; }}")
        elif name == "SUB":
            e(f"    {{ const float g = {g}; a{a} += g; a{b} -= g; }}")
        elif name == "MUL":
            e(f"    {{ const float g = {g}; const float x = v{a}, y = v{b}; a{a} += g * y; a{b} += g * x; }}")
        elif name == "DIV":
            e(f"    {{ const float g = {g}; const float x = v{a}, y = v{b}; a{a} += g / y; a{b} -= g * x / (y * y); }}")
        elif name == "NEG":
            e(f"    a{a} -= {g};")
        elif name == "POWI":
            k = int(b)
            e(f"    {{ const float g = {g}; const float x = v{a}; float p = 1.f;" + " p *= x;" * max(0, k - 1)
              + f" a{a} += g * (float){k} * ({k} > 0 ? p : 0.f); }}")
        elif name == "POWF":
            ex = _lit(consts[b])
            e(f"    {{ const float g = {g}; const float x = v{a}; const float ee = {ex}; a{a} += g * ee * powf(x, ee - 1.f); }}")
        elif name == "SIN":
            e(f"    a{a} += {g} * cosf(v{a});")
        elif name == "COS":
            e(f"    a{a} -= {g} * sinf(v{a});")
        elif name == "EXP":
            e(f"    a{a} += {g} * v{r};")
        elif name == "TANH":
            e(f"    {{ const float t = v{r}; a{a} += {g} * (1.f - t * t); }}")
        elif name == "LOG":
            e(f"    a{a} += {g} / v{a};")
        elif name == "SQRT":
            e(f"    a{a} += {g} * 0.5f / v{r};")
        elif name == "SQUARE":
            e(f"    a{a} += 2.f * {g} * v{a};")


def _group_code(P, gi_meta, n_points, S, d_in, n_terms):
    """Straight-line body of one segment group (mirrors loss_fused_kernel statement by statement)."""
    block_off, phase, n, seg_off, n_slots, loaded = gi_meta
    L = []
    e = L.append
    e(f"    const int i = (blk - {block_off}) * {LF_BLOCK} + tid - {phase};")
    e(f"    const bool active = i >= 0 && i < {n};")
    e("    const int ii = active ? i : 0;")
    nr = max(1, P.n_regs)
    e("    float " + ", ".join(f"v{r}" for r in range(nr)) + ";")
    e("    float " + ", ".join(f"a{r} = 0.f" for r in range(nr)) + ";")

    def load(name, r, a, b):
        return {"STREAM": f"    v{r} = J[(size_t){b} * {n_points} + {seg_off[a]} + ii];",
                "COORD": f"    v{r} = X[(size_t)({seg_off[a]} + ii) * {d_in} + {b}];",
                "VAL": f"    v{r} = ptr.val[{a}][ii];",
                "LAM": f"    v{r} = ptr.lam[{a}][ii];",
                "SCAL": f"    v{r} = *ptr.scal[{a}];"}[name]

    _forward_code(P, e, load)
    for (f, w, t, c) in P.outputs:
        cl = _lit(c)
        e(f"    {{ const float f = v{f}, w = v{w};")
        e(f"      const float contrib = active ? {cl} * w * f * f : 0.f;")
        e("      const float s = block_sum(contrib, red);")
        e(f"      if (tid == 0) acc[{t}] += s;")
        e(f"      if (active) {{ a{f} += 2.f * {cl} * w * f; a{w} += {cl} * f * f; }} }}")

    def store(name, r, a, b, g):
        if name == "STREAM":
            return f"    if (active) dJ[(size_t){b} * {n_points} + {seg_off[a]} + i] = {g};"
        if name == "LAM":
            return f"    if (active) ptr.dlam[{a}][i] = {g};"
        return f"    {{ const float s = block_sum(active ? {g} : 0.f, red); if (tid == 0) acc[{n_terms + a}] += s; }}"

    _reverse_code(P, e, store)
    # dJ of every (point, stream) the program does not read is written as 0
    zero = []
    for sl in range(n_slots):
        for s in range(S):
            if not (loaded[sl] >> s) & 1:
                zero.append(f"dJ[(size_t){s} * {n_points} + {seg_off[sl]} + i] = 0.f;")
    if zero:
        e("    if (active) { " + " ".join(zero) + " }")
    return "\n".join(L)


def generate(op):
    """HIP C++ source of the specialized kernel ``tdq_loss_jit`` for a :class:`.loss_fused.FusedLossOp`."""
    fl, prog = op.fl, op.prog
    S, d_in, N = fl.n_streams, prog.d_in, op.N
    n_terms, n_scal = op.n_terms, op.n_scal
    nacc = n_terms + n_scal
    out = [PRELUDE]
    out.append('extern "C" __global__ void __launch_bounds__(128) tdq_loss_jit(const float* __restrict__ J, '
               'const float* __restrict__ X, float* __restrict__ dJ, float* __restrict__ partials, '
               'const LFPtrs* __restrict__ ptrp, int blk0) {')
    out.append("  __shared__ float red[128 / 16];")
    out.append(f"  __shared__ float acc[{max(1, nacc)}];")
    out.append("  const int tid = threadIdx.x;")
    out.append("  const int blk = blk0 + (int)blockIdx.x;")
    out.append("  const LFPtrs& ptr = *ptrp;")
    out.append(f"  if (tid < {nacc}) acc[tid] = 0.f;")
    for k, (gr, meta) in enumerate(zip(fl.groups, op.group_meta)):
        lo, hi = meta[0], op.group_meta[k + 1][0] if k + 1 < len(op.group_meta) else op.n_blocks
        kw = "if" if k == 0 else "else if"
        out.append(f"  {kw} (blk < {hi}) {{  // group {k}: blocks [{lo}, {hi})")
        out.append(_group_code(gr.program, meta, N, S, d_in, n_terms))
        out.append("  }")
    out.append("  __syncthreads();")
    if nacc:
        out.append(f"  if (tid < {nacc}) partials[(size_t)blk * {nacc} + tid] = acc[tid];")
    out.append("}")
    return "\n".join(out) + "\n"


def device_arch():
    """hipRTC target: the current device's ISA (``gcnArchName`` without feature suffixes), else
    ``TDQ_OFFLOAD_ARCH`` (what ``csrc/build.py`` compiles the library for), else gfx950."""
    try:
        import torch
        if torch.cuda.is_available():
            name = torch.cuda.get_device_properties(torch.cuda.current_device()).gcnArchName
            if name:
                return name.split(":")[0]
    except Exception:  # noqa: BLE001 - fall through to the build setting
        pass
    return os.environ.get("TDQ_OFFLOAD_ARCH", "gfx950")


class LossKernel:
    """A compiled specialized loss kernel (module + function handle), launched like the
    interpreter over any block range."""

    def __init__(self, src, arch=None):
        lib = _lib.load(required=True)
        arch = arch or device_arch()
        key = hashlib.sha256((arch + src).encode()).hexdigest()
        if key not in _CACHE:
            code, size = ctypes.c_void_p(0), ctypes.c_longlong(0)
            log = ctypes.create_string_buffer(8192)
            rc = lib.tdq_rtc_compile(src.encode(), b"tdq_loss_jit.hip", arch.encode(), ctypes.byref(code),
                                     ctypes.byref(size), log, len(log))
            if rc != 0:
                raise RuntimeError(f"hipRTC compile failed ({rc}): {log.value.decode(errors='replace')[:2000]}")
            try:
                mod, fn = ctypes.c_void_p(0), ctypes.c_void_p(0)
                _lib.check(lib.tdq_rtc_load(code, b"tdq_loss_jit", ctypes.byref(mod), ctypes.byref(fn)),
                           "hipModuleLoadData")
            finally:
                lib.tdq_rtc_free(code)
            _CACHE[key] = (mod, fn)
        self.lib = lib
        self.module, self.func = _CACHE[key]

    def launch(self, J, X, dJ, partials, ptrs, blk0, nblk, stream):
        rc = self.lib.tdq_loss_jit_range(self.func, _lib.ptr(J), _lib.ptr(X), _lib.ptr(dJ), _lib.ptr(partials),
                                         _lib.ptr(ptrs), int(blk0), int(nblk), stream)
        _lib.check(rc, "tdq_loss_jit_range")


def compile_for(op):
    """Specialized kernel for ``op`` or ``None`` (disabled, CPU, or any failure - with a warning)."""
    if not enabled() or op.prog.device.type != "cuda":
        return None
    try:
        return LossKernel(generate(op))
    except Exception as e:  # noqa: BLE001 - the interpreter serves every program
        warnings.warn(f"fused loss JIT unavailable, using the interpreter: {type(e).__name__}: {e}")
        return None
