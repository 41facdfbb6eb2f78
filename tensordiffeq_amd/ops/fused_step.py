"""One-launch training step: forward -> loss -> backward of every point (hipRTC).

The persistent point-tile kernel of ``csrc/jet_fused.h`` in its MODE 2 runs, per 32-point tile,
the Taylor-jet forward of the network, the per-point loss of the fused loss program and its
reverse sweep, and the recompute backward into the tile loop's register-resident weight gradient -
so J and dJ never touch HBM and the step has no forward / loss / backward launch boundaries.  The
loss is the traced program of the fused loss (:mod:`.loss_jit` emits the same statements, here as
the body of a ``GenLoss::eval`` the kernel calls per point: every loss group, with the two points
of a periodic pair side by side in the tile), so the kernel is compiled at run time with hipRTC
once per (network shape, loss program) and cached per process.  A step is then the fused launch
plus the two-launch step tail (``jet_hip.step_tail`` / ``dp_tail_a``: slab reduction, loss
bookkeeping, Adam).

Programs with order-3/4 boundary streams (``jet_hi.hip``) run only their residual group fused and
keep the boundary chain (high-order streams, saved-activation forward range, loss blocks, backward
range) on a side stream beside it.

The reference's step is tensordiffeq/models.py:90-135 (``train_op_inner`` / ``update_loss``): a
tape over the network, the residual and the boundary MSEs, then the optimizer.

Precision ``bf16x3`` (the L-BFGS objective) runs the same one-launch structure with every GEMM
operand split into bf16 hi + lo (``csrc/jet_fused3.h``: 16-point tiles, since the lo planes double
the LDS images); its tail reduces fp32 slab rows.

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
_HEADERS = ("common.h", "jet_common.h", "jet_bf3.h", "jet_fused.h", "jet_fused3.h")
# the library's hipcc flags (csrc/build.py _flags), as hipRTC options
RTC_OPTS = "-O3 -std=c++17 -fno-slp-vectorize -munsafe-fp-atomics"


# the bf16x3 objective's kernel under LLVM's max-ILP machine scheduler: 273.3-274.8 vs 277.3-278.2 us
# per evaluation, L-BFGS 0.3190 vs 0.3220 ms per iteration; the bf16 step is faster on the default
# scheduler (0.1378 vs 0.1421 ms) - profiles/r6ba_sched_strategy_ab.txt
# (and col4_sum on ds_bpermute there: the v_permlane swap form is 0.4 % faster in the bf16 step but
# 0.8 % slower in this kernel, profiles/r6be_col4_permlane_ab.txt)
RTC_OPTS_LO = " -mllvm -amdgpu-sched-strategy=max-ilp -DTDQ_COL4_BPERMUTE"


def _opts(src=""):
    """hipRTC options; ``TDQ_FUSED_STEP_TIMING=1`` adds the phase stamps (tools/fused_step_timing.py)."""
    extra = os.environ.get("TDQ_FUSED_STEP_DEFINES", "")   # A/B builds, e.g. "-DTDQ_PK_TANH=0"
    return RTC_OPTS + (RTC_OPTS_LO if "fz3_body<" in src else "") + \
        (" -DTDQ_PHASE_TIMING" if os.environ.get("TDQ_FUSED_STEP_TIMING") == "1" else "") + \
        (" " + extra if extra else "")


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


def spec_source(spec, S, d_in):
    """``SPEC`` / ``DIN`` members of the generated struct: the plan's stream spec (csrc
    jet_common.h ``make_spec``) and the input width as compile-time constants, so the kernel's
    one-hot stream selects and first-layer loops fold away (the kernels require them)."""
    if spec is None or d_in is None:
        raise ValueError("gen_loss: the stream spec and d_in are compile-time constants of the kernel")
    M = 8   # TDQ_MAXS
    st, var, ia, ib = [0] * M, [0] * M, [0] * M, [0] * M
    selA = [[0.0] * M for _ in range(M)]
    selB = [[0.0] * M for _ in range(M)]
    for s in range(S):
        ty, a, b = spec[3 * s:3 * s + 3]
        st[s] = ty
        if ty == 1:
            var[s] = a
        if ty == 2:
            ia[s], ib[s] = a, b
            selA[s][a] = 1.0
            selB[s][b] = 1.0
    arr = lambda v: "{" + ", ".join(str(x) for x in v) + "}"  # noqa: E731
    mat = lambda m: "{" + ", ".join("{" + ", ".join(f"{x:.1f}f" for x in r) + "}" for r in m) + "}"  # noqa: E731
    return [f"  static constexpr JetSpec SPEC = {{{arr(st)}, {arr(var)}, {mat(selA)}, {mat(selB)}, {arr(ia)}, "
            f"{arr(ib)}}};",
            f"  static constexpr int DIN = {int(d_in)};"]


def gen_loss(groups, n_terms, nacc, S, spec=None, d_in=None):
    """``struct GenLoss`` of the loss groups laid out in the fused point set.  ``groups``: one
    ``(program, start, n_slots, n)`` per group - its ``n`` instances occupy points ``start + k``
    (one slot) or the pairs ``start + 2k, start + 2k + 1`` (two slots: a periodic pair side by side,
    ``start`` even, so a pair never straddles a tile of 16 or 32 points).  The statements are those
    of :func:`.loss_jit._group_code` per point: J streams / coordinates from the tile (the partner's
    from the next point-thread), per-point inputs (SA weights, data values, scalars) from global
    memory, loss / scalar-gradient sums into the thread's accumulators, dJ of the instance's points
    into the tile's ``ubs``.  Points outside every group get dJ = 0.  ``eval<S, PT>`` serves both
    tile sizes (``PT`` points per tile)."""
    L = []
    e = L.append
    e("struct GenLoss {")
    e(f"  static constexpr int NACC = {max(1, nacc)};")
    for ln in spec_source(spec, S, d_in):
        e(ln)

    def branches(body):
        kw = "if"
        for (P, start, ns, n) in groups:
            end = start + ns * n
            e(f"    {kw} (n >= {start} && n < {end} && n < N) {{")
            kw = "else if"
            if ns == 2:
                e(f"      if ((n - {start}) & 1) return;   // the pair's first point-thread owns it")
                e(f"      const int i = (n - {start}) >> 1;")
            else:
                e(f"      const int i = n - {start};")
            body(P, ns)
            e("      return;")
            e("    }")

    # the first per-point global input (SA weight / data value) of each group: the kernel loads it
    # for the NEXT tile during this one (pre, into an LDS word per point) - the loss phase then
    # waits for no global load on the common groups (bf16 step 0.1397 -> 0.1382 ms, objective
    # 278.2 -> 277.0 us: profiles/r6ae_loss_input_prefetch_ab.txt)
    first = {}
    for gi, (P, start, ns, n) in enumerate(groups):
        seen = []

        def probe(name, r, a, b, seen=seen):
            if name in ("VAL", "LAM") and not seen:
                seen.append((name, a))
            return ""
        loss_jit._forward_code(P, lambda _ln: None, probe)
        first[gi] = seen[0] if seen else None
    e("  __device__ static float pre(int n, int N, const FzLossPtrs& ptr) {")
    kw = "if"
    for gi, (P, start, ns, n) in enumerate(groups):
        if first[gi] is None:
            continue
        nm, a = first[gi]
        arr = {"VAL": "val", "LAM": "lam"}[nm]
        end = start + ns * n
        idx = f"(n - {start}) >> 1" if ns == 2 else f"n - {start}"
        e(f"    {kw} (n >= {start} && n < {end} && n < N) return ptr.{arr}[{a}][{idx}];")
        kw = "else if"
    e("    return 0.f;")
    e("  }")
    e("  template <int S, int PT, int NW>")
    e("  __device__ static void eval(const float* jv, const float* xs, int t, int n, int N, "
      "const FzLossPtrs& ptr, float* ubs, float (&acc)[NACC], float pv, float bo) {")
    # J of (stream, point): the NW waves' partial output dots summed here (wave order, + bo on the
    # value stream) instead of in a separate phase behind one more barrier
    e("    #define JV(s_, k_) fz_jsum<S, PT, NW>(jv, (s_), (k_), bo)")
    e("    #define UB(s_, k_) ubs[((s_) * PT + (k_)) * 4]")

    cur = {}

    def eval_body(P, ns):
        fp = first[[g[0] for g in groups].index(P)]
        cur["first"], cur["used"] = fp, False
        nr = max(1, P.n_regs)
        e("      float " + ", ".join(f"v{r}" for r in range(nr)) + ";")
        e("      float " + ", ".join(f"a{r} = 0.f" for r in range(nr)) + ";")
        e("      float " + ", ".join(f"dj{sl}_{b} = 0.f" for sl in range(ns) for b in range(S)) + ";")

        def load(name, r, a, b):
            if name in ("STREAM", "COORD") and a >= ns:
                raise ValueError("fused step: slot outside the group")
            if name == "STREAM":
                return f"      v{r} = JV({b}, t + {a});"
            if name == "COORD":
                return f"      v{r} = xs[(t + {a}) * TDQ_MAXD + {b}];"
            if (name, a) == cur["first"] and not cur["used"]:
                cur["used"] = True
                return f"      v{r} = pv;   // prefetched (pre)"
            return {"VAL": f"      v{r} = ptr.val[{a}][i];", "LAM": f"      v{r} = ptr.lam[{a}][i];",
                    "SCAL": f"      v{r} = *ptr.scal[{a}];"}[name]

        loss_jit._forward_code(P, e, load)
        for (f, w, tt, c) in P.outputs:
            cl = loss_jit._lit(c)
            e(f"      {{ const float f = v{f}, w = v{w};")
            e(f"        acc[{tt}] += {cl} * w * f * f;")
            e(f"        a{f} += 2.f * {cl} * w * f; a{w} += {cl} * f * f; }}")

        def store(name, r, a, b, g):
            if name == "STREAM":
                if b >= S:
                    raise ValueError("fused step: stream outside the jet plan")
                return f"      dj{a}_{b} += {g};"
            if name == "LAM":
                return f"      ptr.dlam[{a}][i] = {g};"
            return f"      acc[{n_terms + a}] += {g};"

        loss_jit._reverse_code(P, e, store)
        e("      " + " ".join(f"UB({b}, t + {sl}) = dj{sl}_{b};" for sl in range(ns) for b in range(S)))

    branches(eval_body)
    e("    #pragma unroll")
    e("    for (int s = 0; s < S; ++s) UB(s, t) = 0.f;")
    e("    #undef JV")
    e("    #undef UB")
    e("  }")
    e("};")
    return "\n".join(L)


def kernel_name(lo=False):
    """``tdq_fused_step`` (bf16 step) / ``tdq_fused_step3`` (bf16x3 objective): distinct names in
    the kernel traces."""
    return "tdq_fused_step3" if lo else "tdq_fused_step"


def kernel_source(S, nso, LM, lds, gen, lo=False):
    """The kernel translation unit: the headers, the generated loss, and ``tdq_fused_step`` over
    ``fz_body`` (bf16, 32-point tiles) or ``fz3_body`` (``lo``: bf16x3, 16-point tiles)."""
    body = "fz3_body" if lo else "fz_body"
    return (header_source() + "\n" + gen + "\n"
            'extern "C" __global__ void __launch_bounds__(64 * FZ_WAVES) '
            f"__attribute__((amdgpu_waves_per_eu(2, 2))) {kernel_name(lo)}(FzParams P) {{\n"
            f"  __shared__ __attribute__((aligned(16))) char lds[{lds}];\n"
            f"  {body}<8, {S}, {nso}, {LM}, GenLoss>(P, lds);\n"
            "}\n")


_PENDING = {}   # source key -> (thread, [code bytes | exception])


def _key(src):
    return hashlib.sha256((loss_jit.device_arch() + _opts(src) + src).encode()).hexdigest()


def _rtc_compile(src):
    """hipRTC compile of ``src`` to code-object bytes (host only: no GPU call)."""
    lib = _lib.load(required=True)
    code, size = ctypes.c_void_p(0), ctypes.c_longlong(0)
    log = ctypes.create_string_buffer(16384)
    rc = lib.tdq_rtc_compile_ex(src.encode(), b"tdq_fused_step.hip", loss_jit.device_arch().encode(),
                                _opts(src).encode(), ctypes.byref(code), ctypes.byref(size), log, len(log))
    if rc != 0:
        raise RuntimeError(f"hipRTC compile failed ({rc}): {log.value.decode(errors='replace')[:2000]}")
    try:
        return ctypes.string_at(code, size.value)
    finally:
        lib.tdq_rtc_free(code)


def compile_async(src):
    """Start the hipRTC compile of ``src`` on a host thread (ctypes releases the GIL), so a later
    :func:`_compile` of the same source only loads the module.  No-op when it is cached or pending."""
    import threading
    k = _key(src)
    if k in _CACHE or k in _PENDING:
        return
    out = []

    def work():
        try:
            out.append(_rtc_compile(src))
        except Exception as e:  # noqa: BLE001 - re-raised by _compile
            out.append(e)
    th = threading.Thread(target=work, name="tdq-rtc", daemon=True)
    _PENDING[k] = (th, out)
    th.start()


def _compile(src, name="tdq_fused_step"):
    """``(module, function)`` of the fused-step kernel ``name`` in ``src`` (compiled once per
    process; a compile started by :func:`compile_async` is joined)."""
    lib = _lib.load(required=True)
    k = _key(src)
    if k not in _CACHE:
        pend = _PENDING.pop(k, None)
        if pend is not None:
            pend[0].join()
            code = pend[1][0]
            if isinstance(code, Exception):
                raise code
        else:
            code = _rtc_compile(src)
        buf = ctypes.create_string_buffer(code, len(code))
        mod, fn = ctypes.c_void_p(0), ctypes.c_void_p(0)
        _lib.check(lib.tdq_rtc_load(buf, name.encode(), ctypes.byref(mod), ctypes.byref(fn)), "hipModuleLoadData")
        _CACHE[k] = (mod, fn)
    return _CACHE[k]


def prebuild(prog):
    """Start compiling the fused step of a single-plan program in the background (the L-BFGS
    objective while the Adam phase runs: its hipRTC compile, ~0.35 s, then overlaps the Adam
    steps).  Returns whether a compile was started (or was already cached)."""
    if not torch.cuda.is_available():
        return False
    fop = getattr(prog, "fused_op", None)
    if ineligible(prog, fop) is not None or _mixed(prog):
        return False
    lib = _lib.load()
    cfg = hip_config(prog.net, prog.plan, prog.precision)
    S = cfg["S"]
    spec = jet_hip.stream_spec(prog.plan)
    nso = sum(1 for s in range(S) if spec[3 * s] == 2)
    lo = cfg["precision"] == "bf16x3"
    lds = lib.tdq_jet_fused_lds(cfg["d_in"], jet_hip._warg(cfg), cfg["d_out"], cfg["n_hidden"], S, int(lo))
    gen = gen_loss(_plain_layout(fop.fl), fop.n_terms, fop.n_terms + fop.n_scal, S, spec=spec, d_in=cfg["d_in"])
    compile_async(kernel_source(S, nso, cfg["n_hidden"] - 1, lds, gen, lo=lo))
    return True


def _plain_layout(fl):
    """``[(program, start, n_slots, n)]`` of the fused point set of a single-plan program: groups
    in program order, pair groups on even offsets."""
    layout, pos = [], 0
    for gr in fl.groups:
        ns = len(gr.segs)
        if ns == 2 and pos % 2:
            pos += 1
        layout.append((gr.program, pos, ns, gr.n))
        pos += ns * gr.n
    return layout


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
    if cfg["precision"] not in ("bf16", "bf16x3") or not jet_hip.is_split_bf16(cfg):
        return f"precision {cfg['precision']}"
    lo = cfg["precision"] == "bf16x3"
    if cfg["d_out"] != 1:
        return "d_out != 1"
    lib = _lib.load()
    if lib.tdq_jet_fused_lds(cfg["d_in"], jet_hip._warg(cfg), cfg["d_out"], cfg["n_hidden"], cfg["S"], int(lo)) < 0:
        return f"network {cfg['widths']} / S={cfg['S']} (width-128 MFMA layers 2-3, S <= 4)"
    fl = fop.fl
    for gr in fl.groups:
        if any(s >= cfg["S"] for (_, s) in gr.program.stream_regs) and not _mixed(prog):
            return "a loss group reads streams outside the jet plan"
    mode = _mixed_mode(prog)
    if mode is not None and lo:
        # the bf16x3 objective of a mixed program keeps the point-range launches (its boundary
        # chain runs on the bf16x3 jet_hi kernels beside them)
        return "bf16x3: high-order boundary streams keep the separate launches"
    if mode == "0":
        return "high-order boundary streams (TDQ_FUSED_STEP_MIXED=0)"
    if mode == "split":
        sp = _split_groups(prog, fop, cfg["S"])
        return sp if isinstance(sp, str) else None
    if mode == "1":
        # high-order boundary points (jet_hi.hip streams): only the residual group runs fused
        last = len(prog.segments) - 1
        gr = fl.groups[-1]
        if gr.segs != [last] or any(last in g.segs for g in fl.groups[:-1]):
            return "the last segment is not a group of its own"
        if any(s >= cfg["S"] for (_, s) in gr.program.stream_regs):
            return "the residual loss reads streams outside the jet plan"
        seg = prog.segments[last]
        if seg.offset + gr.n != prog.X_all.shape[0]:
            return "the residual segment does not end the point set"
        if prog.n_hi > seg.offset:
            return "high-order points inside the residual segment"
    return None


def _mixed(prog):
    return getattr(prog, "hi_op", None) is not None


def _mixed_mode(prog):
    """Layout of a mixed program (order-3/4 boundary streams from jet_hi.hip), ``TDQ_FUSED_STEP_MIXED``:
    ``split`` (default) - every loss output on main-plan streams runs in the fused launch (the
    boundary groups' low-order outputs included), only the high-order outputs' chain (jet_hi
    forward, their loss blocks, jet_hi adjoint) on a side stream; ``1`` - only the residual group
    fused, the whole boundary chain on the side stream; ``0`` - the point-range path.  MI355X,
    AC-baseline 50k: split 0.207 ms/step, residual 0.251, point ranges 0.219-0.226 (AC-SA 0.168;
    profiles/r5split3_*, r5acb_*).  None: not mixed."""
    if not _mixed(prog):
        return None
    return os.environ.get("TDQ_FUSED_STEP_MIXED", "split")


def _split_groups(prog, fop, S):
    """``[(group, fused program, side program or None)]`` of the split layout, or the reason it
    does not apply (an output reading main-plan and high-order streams together, or an SA weight
    read by both halves)."""
    from .. import fusion
    out = []
    for gr in fop.fl.groups:
        if all(s < S for (_, s) in gr.program.stream_regs):
            out.append((gr, gr.program, None))
            continue
        sp = fusion.split_by_streams(fop.fl, gr, S)
        if sp is None:
            return "a loss output reads main-plan and high-order streams together (or both read one SA weight)"
        out.append((gr, sp[0], sp[1]))
    return out


class FusedStepOp:
    """The fused training step of a :class:`~tensordiffeq_amd.models.loss.LossProgram` (built by
    :func:`for_program`).

    Single-plan programs: EVERY loss group runs in the one launch - the points re-laid out once
    into a fused point set (each group's instances contiguous, a periodic group's two segments
    interleaved pair by pair), so a step is the fused launch + the two-launch step tail.  Precision
    bf16: 32-point tiles (``jet_fused.h``); bf16x3 (the L-BFGS objective): 16-point tiles with hi +
    lo operands (``jet_fused3.h``) and fp32 slab rows.  Mixed programs (order-3/4 boundary streams
    from jet_hi.hip, bf16 only, :func:`_mixed_mode`): split layout - every loss output on main-plan
    streams in the fused launch, the high-order outputs (their own loss op,
    :func:`fusion.split_by_streams`) with the jet_hi forward / adjoint on a side stream beside it;
    residual layout - the residual group fused over its own segment, the whole boundary chain
    (high-order streams, saved-activation forward, loss blocks, backward) on the side stream."""

    def __init__(self, prog, fop):
        lib = _lib.load(required=True)
        self.prog, self.fop = prog, fop
        cfg = self.cfg = hip_config(prog.net, prog.plan, prog.precision)
        self.lo = cfg["precision"] == "bf16x3"
        self.pt = 16 if self.lo else 32
        fl = fop.fl
        S = cfg["S"]
        self.nacc = fop.n_terms + fop.n_scal
        spec = jet_hip.stream_spec(prog.plan)
        nso = sum(1 for s in range(S) if spec[3 * s] == 2)
        LM = cfg["n_hidden"] - 1
        lds = lib.tdq_jet_fused_lds(cfg["d_in"], jet_hip._warg(cfg), cfg["d_out"], cfg["n_hidden"], S, int(self.lo))
        if lds < 0 or lds > 160 * 1024:
            raise ValueError(f"fused step: {lds} bytes of LDS")
        self.lds = lds
        N = prog.X_all.shape[0]
        dev = prog.device
        self.mixed = _mixed(prog)
        self.layout = "plain" if not self.mixed else ("split" if _mixed_mode(prog) == "split" else "residual")
        self.fop2 = None
        if self.layout != "residual":
            # the fused point set: groups in program order, pair groups on even offsets (split
            # layout: the boundary groups with their main-plan outputs only)
            groups = [(gr, gr.program, None) for gr in fl.groups] if not self.mixed else _split_groups(prog, fop, S)
            layout, idx, pos = [], [], 0
            for gr, P_f, _ in groups:
                ns = len(gr.segs)
                if ns == 2 and pos % 2:
                    idx.append(-1)
                    pos += 1
                layout.append((P_f, pos, ns, gr.n))
                offs = [prog.segments[sg].offset for sg in gr.segs]
                for k in range(gr.n):
                    idx.extend(o + k for o in offs)
                pos += ns * gr.n
            ix = torch.tensor(idx, dtype=torch.long, device=dev)
            X_f = prog.X_all[ix.clamp_min(0)].clone()
            X_f[ix < 0] = 0.0
            self.X = X_f.contiguous()
            self.N, self.p_lo, self.srow, self.b_res, self.p_bc, self.seg_lo = pos, 0, 0, 0, 0, 0
            if self.layout == "split":
                # the high-order outputs: a loss op of their own (same term / value / lambda / scalar
                # slots - its pointer table is the main op's), its block rows ahead of the fused rows
                import copy
                from ..fusion import Group
                from .loss_fused import FusedLossOp
                fl2 = copy.copy(fl)
                fl2.groups = []
                for gr, _, P_s in groups:
                    if P_s is not None:
                        g2 = Group(list(gr.segs), gr.n)
                        g2.program = P_s
                        fl2.groups.append(g2)
                self.fop2 = FusedLossOp(fl2, prog, fop.lams, fop.scalars, fl.lam_offsets)
                self.fop2.ptrs = fop.ptrs
                self.b_res = self.fop2.n_blocks
        else:
            self.seg_lo = prog.segments[-1].offset
            layout = [(fl.groups[-1].program, self.seg_lo, 1, fl.groups[-1].n)]
            self.X = None                               # the program's X_all
            self.N, self.p_lo = N, self.seg_lo
            self.b_res = fop.group_meta[-1][0]          # the residual group's first loss block
            # boundary points: the saved-activation chain over [0, p_bc) - its backward workgroups
            # own slab rows [0, srow); points [seg_lo, p_bc) ride along with dJ = 0
            pts_b = jet_hip.slab_geometry(cfg, N)[0]
            self.p_bc = min(N, -(-self.seg_lo // 128) * 128) if self.seg_lo > 0 else 0
            self.srow = -(-self.p_bc // pts_b)
        self.source = kernel_source(S, nso, LM, lds, gen_loss(layout, fop.n_terms, self.nacc, S, spec=spec,
                                                              d_in=cfg["d_in"]), lo=self.lo)
        self.module, self.func = _compile(self.source, kernel_name(self.lo))
        ntiles = -(-(self.N - self.p_lo) // self.pt)
        cus = max(1, lib.tdq_device_cus())
        rounds = -(-ntiles // cus)
        if self.fop2 is not None:
            # split layout: one round more leaves ~57 CUs to the jet_hi side chain - AC-baseline 50k
            # (7 rounds) 0.2070 vs 0.2105 ms/step (+2 rounds: 0.2277), profiles/r5split3_*; with many
            # rounds the extra one costs more than the side chain gains - AC-dist 500k (62 rounds)
            # 1.043-1.048 ms/step without it, 1.058-1.060 with it (profiles/r6ao_ac_dist_rounds.txt)
            rounds += int(os.environ.get("TDQ_FS_SPLIT_ROUNDS", "1" if rounds <= 16 else "0"))
        # the fewest workgroups with the same tiles per workgroup (AC-SA 50k, bf16: 1592 tiles,
        # 228 x 7; bf16x3: 3183 tiles, 245 x 13)
        self.G = -(-ntiles // rounds)
        self.free_cus = cus - self.G   # CUs the persistent workgroups leave to a side chain
        if self.layout == "residual":   # the fused rows follow the boundary loss blocks' rows in fop.partials
            self.G = min(self.G, fop.n_blocks - self.b_res)
        self.rows = self.srow + self.G
        need = lib.tdq_slab_floats_rows(self.rows, cfg["d_in"], jet_hip._warg(cfg), cfg["d_out"], cfg["n_hidden"])
        cap = lib.tdq_jet_bf3_slab_floats(N, cfg["d_in"], jet_hip._warg(cfg), cfg["d_out"], cfg["n_hidden"])
        if need < 0 or need > cap:
            raise ValueError(f"fused step: {self.rows} slab rows do not fit the backward's buffer")
        # loss partials: the boundary loss blocks' rows (mixed) then one row per fused workgroup
        self.n_lblocks = self.b_res + self.G
        self.lpart = torch.zeros(max(1, self.n_lblocks * self.nacc), dtype=torch.float32, device=dev)
        if self.fop2 is not None:   # the side chain's loss blocks write rows [0, b_res) of the same buffer
            self.fop2.partials = self.lpart[:self.b_res * self.nacc]
        self._side = torch.cuda.Stream(device=dev) if (self.p_bc > 0 or self.fop2 is not None) else None

    def run(self, saved, J, work, flat, pack=True):
        """The step's gradient slabs and loss partials (the fused launch; mixed programs: plus the
        boundary chain on a side stream, joined before return).  ``saved`` / ``J`` / ``work``: the
        persistent step buffers of ``jet_hip.alloc_forward`` / ``alloc_backward``."""
        lib = _lib.load()
        fop, cfg = self.fop, self.cfg
        if pack:
            jet_hip.pack_images(saved)
        cur = torch.cuda.current_stream(flat.device)
        side = self._side
        hop = self.prog.hi_op
        X, _, scratch, _, spec, S = saved
        spec_arr = (ctypes.c_int * len(spec))(*spec)
        Xf = self.X if self.X is not None else X
        lpart = fop.partials if self.layout == "residual" else self.lpart

        def boundary():
            if self.fop2 is not None:   # split layout: only the high-order outputs' chain
                hop.forward(J, flat)
                self.fop2.run_range(J, 0, self.fop2.n_blocks)
                hop.backward(self.fop2.dJ, flat)
                return
            hop.forward(J, flat)
            jet_hip.forward_range(saved, J, 0, self.p_bc)
            if self.b_res > 0:
                fop.run_range(J, 0, self.b_res)
            hop.backward(fop.dJ, flat)
            if self.p_bc > self.seg_lo:
                fop.dJ[:, self.seg_lo:self.p_bc].zero_()
            jet_hip.backward_range(saved, fop.dJ, work, 0, self.p_bc)

        def fused():
            rc = lib.tdq_fused_step_launch(self.func, _lib.ptr(Xf), _lib.ptr(scratch), _lib.ptr(work), self.N,
                                           cfg["d_in"], jet_hip._warg(cfg), cfg["d_out"], cfg["n_hidden"], S,
                                           spec_arr, self.p_lo, self.srow, self.G, _lib.ptr(fop.ptrs),
                                           _lib.ptr(lpart), self.b_res, self.nacc, int(self.lo),
                                           _lib.stream_ptr(flat.device))
            _lib.check(rc, "tdq_fused_step_launch")

        if side is None:
            fused()
            return
        # split layout: which branch is captured first.  With >= 32 CUs left to the side chain
        # (AC-baseline 50k: 56) the fused launch goes first and no longer starts ~11 us into the step
        # behind the fork: 0.1638 vs 0.1736 ms/step (profiles/r6aj_ac_baseline_split_order.txt).
        # With few free CUs (AC-dist 500k: 7) the jet_hi forward launched second waited for the whole
        # fused launch (964 us) and the chain ran after it (profiles/r6am_*): side chain first
        order = os.environ.get("TDQ_FS_SPLIT_ORDER", "fused_first" if self.free_cus >= 32 else "side_first")
        if self.fop2 is not None and order == "side_first":
            ev = torch.cuda.Event()
            ev.record(cur)
            side.wait_event(ev)
            with torch.cuda.stream(side):
                boundary()
            fused()
            cur.wait_stream(side)
            return
        # the fused launch is the graph's first node and the boundary branch forks from before it:
        # MI355X, AC-SA (side chain layout): 0.1697 vs 0.1813 ms/step with the branch captured
        # first (profiles/r5ord_*: the fused kernel then started ~6 us later and the join waited
        # ~10 us on the other queue)
        ev = torch.cuda.Event()
        ev.record(cur)
        fused()
        side.wait_event(ev)
        with torch.cuda.stream(side):
            boundary()
        cur.wait_stream(side)

    def set_timing_buffer(self, buf):
        """Phase-stamp build only: the int64 buffer of the stamps ([G * 8 waves][64])."""
        _lib.check(_lib.load().tdq_rtc_set_global_ptr(self.module, b"tdq_ts", ctypes.c_void_p(buf.data_ptr())),
                   "tdq_rtc_set_global_ptr")

    def tail_kw(self):
        """Keyword arguments of ``jet_hip.step_tail`` / ``dp_tail_a`` for this step's rows (the slab
        precision follows the program's: bf16 rows for bf16, fp32 rows for bf16x3)."""
        return {"rows": self.rows, "lpart": self.fop.partials if self.layout == "residual" else self.lpart,
                "n_lblocks": self.n_lblocks}


def for_program(prog):
    """The program's :class:`FusedStepOp` (built once), or ``None`` (reason in
    ``prog.fused_step_reason``)."""
    if getattr(prog, "_fused_step_built", False):
        return prog._fused_step
    if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
        # module loads cannot run inside a capture: the engines build the op before capturing
        # (fit.AdamEngine._capture, the L-BFGS drivers' first eager evaluation) - never cache a
        # "not available" decided here
        warnings.warn("fused training step first requested inside a graph capture; using separate launches")
        return None
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
