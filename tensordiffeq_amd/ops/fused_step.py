"""One-launch training step of the residual points: forward -> loss -> backward (hipRTC).

The persistent point-tile kernel of ``csrc/jet_fused.h`` in its MODE 2 runs, per 32-point tile,
the Taylor-jet forward of the network, the residual group's per-point loss and its reverse sweep,
and the recompute backward into the tile loop's register-resident weight gradient - so the residual
points' J and dJ never touch HBM and the step has no forward / loss / backward launch boundaries.
The loss is the traced program of the fused loss (:mod:`.loss_jit` emits the same statements, here
as the body of a ``GenLoss::eval`` the kernel calls per point), so the kernel is compiled at run
time with hipRTC once per (network shape, loss program) and cached per process.

The boundary / initial points (the groups before the residual segment) keep the saved-activation
chain of ``csrc/jet_bf3.h`` (forward range -> loss blocks -> backward range) on a side stream beside
the fused launch, which leaves them CUs (``FusedStepOp.G``); the fused step tail
(``jet_hip.step_tail`` / ``dp_tail_a``) then reduces both sets of gradient-slab rows and loss
partials and runs Adam.

The reference's step is tensordiffeq/models.py:90-135 (``train_op_inner`` / ``update_loss``): a
tape over the network, the residual and the boundary MSEs, then the optimizer - here one fused
launch for the 98% of points that are residual points.

``TDQ_FUSED_STEP=0`` keeps the separate launches (``fit.run_ranges``).
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import warnings

import torch

from . import _lib, jet_hip, loss_jit
from .jet_mlp import hip_config

_CACHE = {}   # source sha -> (module, func)
_HEADERS = ("common.h", "jet_common.h", "jet_bf3.h", "jet_fused.h")
# the library's hipcc flags (csrc/build.py _flags), as hipRTC options
RTC_OPTS = "-O3 -std=c++17 -fno-slp-vectorize -munsafe-fp-atomics"


def enabled():
    return os.environ.get("TDQ_FUSED_STEP", "1") != "0"


def _csrc():
    return os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc")


def header_source():
    """The kernel headers as one translation unit (hipRTC has no include path of ours)."""
    out = []
    for h in _HEADERS:
        with open(os.path.join(_csrc(), h)) as f:
            lines = f.read().splitlines()
        out.append("\n".join(ln for ln in lines if not ln.strip().startswith('#include "')
                             and ln.strip() != "#pragma once"))
    return "\n".join(out)


def gen_loss(P, n_terms, nacc):
    """``struct GenLoss`` of one single-segment group program: the loss statements of
    :func:`.loss_jit._group_code` per point (J streams and coordinates from the kernel's registers,
    loss / scalar-gradient sums into the thread's accumulators, dJ into ``dJv``)."""
    L = []
    e = L.append
    nr = max(1, P.n_regs)
    e("struct GenLoss {")
    e(f"  static constexpr int NACC = {max(1, nacc)};")
    e("  template <int S>")
    e("  __device__ static void eval(const float (&Jv)[S], const float* xr, int i, bool active, "
      "const FzLossPtrs& ptr, float (&dJv)[S], float (&acc)[NACC]) {")
    e("    const int ii = active ? i : 0;")
    e("    #pragma unroll")
    e("    for (int s = 0; s < S; ++s) dJv[s] = 0.f;")
    e("    float " + ", ".join(f"v{r}" for r in range(nr)) + ";")
    e("    float " + ", ".join(f"a{r} = 0.f" for r in range(nr)) + ";")

    def load(name, r, a, b):
        if name in ("STREAM", "COORD") and a != 0:
            raise ValueError("fused step: the residual group reads one segment")
        return {"STREAM": f"    v{r} = Jv[{b}];",
                "COORD": f"    v{r} = xr[{b}];",
                "VAL": f"    v{r} = ptr.val[{a}][ii];",
                "LAM": f"    v{r} = ptr.lam[{a}][ii];",
                "SCAL": f"    v{r} = *ptr.scal[{a}];"}[name]

    loss_jit._forward_code(P, e, load)
    for (f, w, t, c) in P.outputs:
        cl = loss_jit._lit(c)
        e(f"    {{ const float f = v{f}, w = v{w};")
        e(f"      acc[{t}] += active ? {cl} * w * f * f : 0.f;")
        e(f"      if (active) {{ a{f} += 2.f * {cl} * w * f; a{w} += {cl} * f * f; }} }}")

    def store(name, r, a, b, g):
        if name == "STREAM":
            return f"    dJv[{b}] += {g};"
        if name == "LAM":
            return f"    if (active) ptr.dlam[{a}][i] = {g};"
        return f"    acc[{n_terms + a}] += active ? {g} : 0.f;"

    loss_jit._reverse_code(P, e, store)
    e("  }")
    e("};")
    return "\n".join(L)


def kernel_source(S, nso, LM, lds, gen):
    return (header_source() + "\n" + gen + "\n"
            'extern "C" __global__ void __launch_bounds__(64 * FZ_WAVES) '
            "__attribute__((amdgpu_waves_per_eu(2, 2))) tdq_fused_step(FzParams P) {\n"
            f"  __shared__ __attribute__((aligned(16))) char lds[{lds}];\n"
            f"  fz_body<8, {S}, {nso}, {LM}, 2, GenLoss>(P, lds);\n"
            "}\n")


def _compile(src):
    lib = _lib.load(required=True)
    arch = loss_jit.device_arch()
    key = hashlib.sha256((arch + RTC_OPTS + src).encode()).hexdigest()
    if key not in _CACHE:
        code, size = ctypes.c_void_p(0), ctypes.c_longlong(0)
        log = ctypes.create_string_buffer(16384)
        rc = lib.tdq_rtc_compile_ex(src.encode(), b"tdq_fused_step.hip", arch.encode(), RTC_OPTS.encode(),
                                    ctypes.byref(code), ctypes.byref(size), log, len(log))
        if rc != 0:
            raise RuntimeError(f"hipRTC compile failed ({rc}): {log.value.decode(errors='replace')[:2000]}")
        try:
            mod, fn = ctypes.c_void_p(0), ctypes.c_void_p(0)
            _lib.check(lib.tdq_rtc_load(code, b"tdq_fused_step", ctypes.byref(mod), ctypes.byref(fn)),
                       "hipModuleLoadData")
        finally:
            lib.tdq_rtc_free(code)
        _CACHE[key] = (mod, fn)
    return _CACHE[key][1]


def ineligible(prog, fop):
    """Why the fused step cannot serve this program (``None``: it can)."""
    if not enabled():
        return "TDQ_FUSED_STEP=0"
    if prog.device.type != "cuda" or fop is None:
        return "needs the fused loss on a GPU"
    try:
        cfg = hip_config(prog.net, prog.plan, prog.precision)
    except ValueError as e:
        return str(e)
    if cfg["precision"] != "bf16" or not jet_hip.is_split_bf16(cfg):
        return f"precision {cfg['precision']}"
    if jet_hip.fused_active(cfg):
        return "TDQ_FUSED=1 (persistent forward / backward launches)"
    if cfg["d_out"] != 1:
        return "d_out != 1"
    lib = _lib.load()
    if lib.tdq_jet_fused_lds(cfg["d_in"], jet_hip._warg(cfg), cfg["d_out"], cfg["n_hidden"], cfg["S"], 2) < 0:
        return f"network {cfg['widths']} / S={cfg['S']} (width-128 MFMA layers 2-3, S <= 4)"
    fl = fop.fl
    last = len(prog.segments) - 1
    gr = fl.groups[-1]
    if gr.segs != [last] or any(last in g.segs for g in fl.groups[:-1]):
        return "the last segment is not a group of its own"
    if any(s >= cfg["S"] for (_, s) in gr.program.stream_regs):
        return "the residual loss reads streams outside the jet plan"
    seg = prog.segments[last]
    if seg.offset + gr.n != prog.X_all.shape[0]:
        return "the residual segment does not end the point set"
    if getattr(prog, "hi_op", None) is not None and prog.n_hi > seg.offset:
        return "high-order points inside the residual segment"
    return None


class FusedStepOp:
    """The fused step of a :class:`~tensordiffeq_amd.models.loss.LossProgram` whose residual group
    is its last segment (built by :func:`for_program`)."""

    def __init__(self, prog, fop):
        lib = _lib.load(required=True)
        self.prog, self.fop = prog, fop
        cfg = self.cfg = hip_config(prog.net, prog.plan, prog.precision)
        N = self.N = prog.X_all.shape[0]
        fl = fop.fl
        self.seg_lo = prog.segments[-1].offset
        self.b_res = fop.group_meta[-1][0]         # the residual group's first loss block
        self.nacc = fop.n_terms + fop.n_scal
        spec = jet_hip.stream_spec(prog.plan)
        S = cfg["S"]
        nso = sum(1 for s in range(S) if spec[3 * s] == 2)
        LM = cfg["n_hidden"] - 1
        lds = lib.tdq_jet_fused_lds(cfg["d_in"], jet_hip._warg(cfg), cfg["d_out"], cfg["n_hidden"], S, 2)
        if lds < 0 or lds > 160 * 1024:
            raise ValueError(f"fused step: {lds} bytes of LDS")
        self.source = kernel_source(S, nso, LM, lds, gen_loss(fl.groups[-1].program, fop.n_terms, self.nacc))
        self.func = _compile(self.source)
        # boundary points: the saved-activation chain over [0, p_bc) - its backward workgroups own
        # slab rows [0, srow); points [seg_lo, p_bc) ride along with dJ = 0
        pts_b = jet_hip.slab_geometry(cfg, N)[0]
        self.p_bc = min(N, -(-self.seg_lo // 128) * 128) if self.seg_lo > 0 else 0
        self.srow = -(-self.p_bc // pts_b)
        ntiles = -(-(N - self.seg_lo) // 32)
        cus = max(1, lib.tdq_device_cus())
        rounds = -(-ntiles // cus)
        # the fewest workgroups with the same tiles per workgroup: the CUs left over run the
        # boundary chain beside the fused launch (AC-SA 50k: 1563 tiles, 224 workgroups x 7)
        self.G = min(-(-ntiles // rounds), fop.n_blocks - self.b_res)
        need = lib.tdq_slab_floats_rows(self.srow + self.G, cfg["d_in"], jet_hip._warg(cfg), cfg["d_out"],
                                        cfg["n_hidden"])
        cap = lib.tdq_jet_bf3_slab_floats(N, cfg["d_in"], jet_hip._warg(cfg), cfg["d_out"], cfg["n_hidden"])
        if self.G < 1 or need < 0 or need > cap:
            raise ValueError(f"fused step: {self.srow + self.G} slab rows do not fit the backward's buffer")
        self.rows = self.srow + self.G
        self.n_lblocks = self.b_res + self.G
        self.lds = lds
        self._side = torch.cuda.Stream(device=prog.device) if self.p_bc > 0 else None

    def run(self, saved, J, work, flat, pack=True):
        """The step's gradient slabs and loss partials: boundary chain on a side stream, the fused
        launch on the current one (joined before return).  ``saved`` / ``J`` / ``work``: the
        persistent step buffers of ``jet_hip.alloc_forward`` / ``alloc_backward``."""
        lib = _lib.load()
        fop, cfg = self.fop, self.cfg
        if pack:
            jet_hip.pack_images(saved)
        cur = torch.cuda.current_stream(flat.device)
        side = self._side
        hop = self.prog.hi_op   # mixed programs: the high-order boundary points' extra streams
        if side is not None:
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                if hop is not None:
                    hop.forward(J, flat)
                jet_hip.forward_range(saved, J, 0, self.p_bc)
                if self.b_res > 0:
                    fop.run_range(J, 0, self.b_res)
                if hop is not None:
                    hop.backward(fop.dJ, flat)
                if self.p_bc > self.seg_lo:
                    fop.dJ[:, self.seg_lo:self.p_bc].zero_()
                jet_hip.backward_range(saved, fop.dJ, work, 0, self.p_bc)
        X, _, scratch, _, spec, S = saved
        spec_arr = (ctypes.c_int * len(spec))(*spec)
        rc = lib.tdq_fused_step_launch(self.func, _lib.ptr(X), _lib.ptr(scratch), _lib.ptr(work), self.N,
                                       cfg["d_in"], jet_hip._warg(cfg), cfg["d_out"], cfg["n_hidden"], S, spec_arr,
                                       self.seg_lo, self.srow, self.G, _lib.ptr(fop.ptrs), _lib.ptr(fop.partials),
                                       self.b_res, self.nacc, self.seg_lo, _lib.stream_ptr(flat.device))
        _lib.check(rc, "tdq_fused_step_launch")
        if side is not None:
            cur.wait_stream(side)

    def tail_kw(self):
        """Keyword arguments of ``jet_hip.step_tail`` / ``dp_tail_a`` for this step's rows."""
        return {"rows": self.rows, "lpart": self.fop.partials, "n_lblocks": self.n_lblocks}


def for_program(prog):
    """The program's :class:`FusedStepOp` (built once), or ``None`` (reason in
    ``prog.fused_step_reason``)."""
    if getattr(prog, "_fused_step_built", False):
        return prog._fused_step
    prog._fused_step_built = True
    prog._fused_step = None
    fop = getattr(prog, "fused_op", None)
    why = ineligible(prog, fop)
    if why is None:
        try:
            prog._fused_step = FusedStepOp(prog, fop)
        except Exception as e:  # noqa: BLE001 - the separate launches serve every program
            why = f"{type(e).__name__}: {e}"
            warnings.warn(f"fused training step unavailable, using separate launches: {why}")
    prog.fused_step_reason = why
    return prog._fused_step
