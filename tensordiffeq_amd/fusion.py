"""Loss fusion: trace user callables into one elementwise program, run it in one HIP kernel.

Why: after the jet kernels, the rest of a training step is elementwise - the PDE residual built
from the jet streams, boundary differences, squares, self-adaptive weighting, means - plus the
adjoints of all of that.  Executed as torch ops that is ~60 tiny kernels per step (and autograd
materialises a zero-filled full-size dJ for every segment slice).  Here every user callable
(``f_model``, ``deriv_model``s, ``g``) is traced ONCE with symbolic values (:class:`Sym`) into a
DAG over the inputs of one collocation point:

  stream(seg, mi)   jet stream ``mi`` of the network output at this point of segment ``seg``
  coord(seg, j)     coordinate j of the point
  val(k)            per-point target value array k (IC / Dirichlet / Neumann / data)
  lam(k)            per-point self-adaptive weight array k
  scal(k)           scalar parameter k (scalar SA weight, DiscoveryModel coefficient)
  const             python / 0-dim tensor constants

Every loss term becomes a set of outputs ``(f, w, term, c)`` contributing ``c * w * f^2`` to
``loss[term]`` (``w`` = 1, lambda^2, g(lambda) or a scalar lambda: one formula covers the
reference's MSE / SA-MSE / g_MSE / outside-sum forms).  The DAG is compiled to a flat bytecode
(SSA registers); ``csrc/loss_fused.hip`` interprets it with one thread per point (registers in
LDS): forward values, losses, reverse-mode adjoints, writes ``dJ`` (every stream of every point
of the group, zeros included), ``dlam`` per point and block partials of losses / scalar
gradients, then a deterministic reduction kernel finishes the sums.  :func:`run_reference`
executes the same bytecode with torch (CPU tests / oracle).

Anything the tracer cannot express (non-elementwise ops, data-dependent Python control flow on
values, multi-output networks) makes :func:`build` return ``None`` and the solver keeps the
autograd-composed loss.
"""
from __future__ import annotations

import math
import numbers

import numpy as np
import torch

from . import autodiff

# opcodes (keep in sync with csrc/loss_fused.hip)
OP = dict(STREAM=1, COORD=2, VAL=3, CONST=4, LAM=5, SCAL=6,
          ADD=10, SUB=11, MUL=12, DIV=13, NEG=14, POWI=15, POWF=16, SIN=17, COS=18, EXP=19,
          TANH=20, LOG=21, SQRT=22, SQUARE=23)
UNARY = {"neg": "NEG", "sin": "SIN", "cos": "COS", "exp": "EXP", "tanh": "TANH", "log": "LOG",
         "sqrt": "SQRT", "square": "SQUARE"}
MAX_REGS = 120


class TraceError(RuntimeError):
    pass


class Graph:
    def __init__(self):
        self.nodes = []      # (kind, args...) ; index = node id
        self.memo = {}

    def add(self, key):
        if key in self.memo:
            return self.memo[key]
        self.nodes.append(key)
        self.memo[key] = len(self.nodes) - 1
        return self.memo[key]


class Sym:
    """Symbolic scalar-per-point value recorded into a :class:`Graph`."""

    __slots__ = ("g", "i")

    def __init__(self, g, i):
        self.g, self.i = g, i

    # -- helpers ------------------------------------------------------------------------
    def _c(self, v):
        if isinstance(v, Sym):
            if v.g is not self.g:
                raise TraceError("mixing traces")
            return v
        if isinstance(v, torch.Tensor):
            if v.numel() != 1:
                raise TraceError("non-scalar tensor constant in a traced expression")
            v = float(v.detach().reshape(()).item())
        if isinstance(v, (numbers.Number, np.floating, np.integer)):
            return Sym(self.g, self.g.add(("const", float(v))))
        raise TraceError(f"unsupported operand {type(v)}")

    def _bin(self, op, o, rev=False):
        o = self._c(o)
        a, b = (o, self) if rev else (self, o)
        return Sym(self.g, self.g.add((op, a.i, b.i)))

    def _un(self, op):
        return Sym(self.g, self.g.add((op, self.i)))

    __add__ = lambda s, o: s._bin("add", o)
    __radd__ = lambda s, o: s._bin("add", o, True)
    __sub__ = lambda s, o: s._bin("sub", o)
    __rsub__ = lambda s, o: s._bin("sub", o, True)
    __mul__ = lambda s, o: s._bin("mul", o)
    __rmul__ = lambda s, o: s._bin("mul", o, True)
    __truediv__ = lambda s, o: s._bin("div", o)
    __rtruediv__ = lambda s, o: s._bin("div", o, True)
    __neg__ = lambda s: s._un("neg")
    __pos__ = lambda s: s

    def __pow__(self, e):
        if isinstance(e, torch.Tensor) and e.numel() == 1:
            e = float(e.item())
        if isinstance(e, Sym):
            raise TraceError("symbolic exponent")
        e = float(e)
        if e == int(e) and 0 <= e <= 16:
            return Sym(self.g, self.g.add(("powi", self.i, int(e))))
        return Sym(self.g, self.g.add(("powf", self.i, e)))

    def __rpow__(self, base):
        return (self * math.log(float(base))).exp()

    def exp(self):
        return self._un("exp")

    def sin(self):
        return self._un("sin")

    def cos(self):
        return self._un("cos")

    def tanh(self):
        return self._un("tanh")

    def log(self):
        return self._un("log")

    def sqrt(self):
        return self._un("sqrt")

    def square(self):
        return self._un("square")

    # shape no-ops (values are per point)
    def reshape(self, *a, **k):
        return self

    view = reshape
    squeeze = reshape
    unsqueeze = reshape
    contiguous = reshape
    float = reshape

    def __getitem__(self, idx):
        return self

    def __getattr__(self, name):
        raise TraceError(f"unsupported tensor method .{name}() in a traced expression")

    def __bool__(self):
        raise TraceError("data-dependent control flow on a traced value")

    @property
    def shape(self):
        return (1, 1)

    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        name = getattr(func, "__name__", str(func)).lstrip("_").rstrip("_")
        syms = [a for a in args if isinstance(a, Sym)]
        if name in ("cat", "stack", "hstack", "concat"):
            return _CatMarker()
        if name in ("ones_like",):  # the unit cotangent of torch.autograd.grad(u, x, ones_like(u))
            return _OnesMarker()
        if not syms:
            raise TraceError(f"unsupported torch function {name}")
        s = syms[0]
        if name in ("add", "radd"):
            return s._c(args[0]) + s._c(args[1]) if len(args) > 1 else s
        if name in ("sub", "rsub"):
            return (s._c(args[0]) - s._c(args[1])) if name == "sub" else (s._c(args[1]) - s._c(args[0]))
        if name in ("mul", "rmul"):
            return s._c(args[0]) * s._c(args[1])
        if name in ("div", "truediv", "true_divide"):
            return s._c(args[0]) / s._c(args[1])
        if name in ("rdiv", "rtruediv"):
            return s._c(args[1]) / s._c(args[0])
        if name in ("pow",):
            if isinstance(args[0], Sym):
                return args[0] ** args[1]
            raise TraceError("symbolic exponent")
        if name == "rpow":
            return args[0].__rpow__(args[1])
        if name in ("neg", "negative"):
            return -s
        if name in UNARY:
            return s._un(name)
        if name in ("reshape", "view", "squeeze", "unsqueeze", "contiguous", "clone", "float"):
            return s
        raise TraceError(f"unsupported torch function {name}")


class _CatMarker:
    """Result of ``torch.cat([x, t], 1)`` inside a traced callable (only fed to u_model)."""


class _OnesMarker:
    """Result of ``torch.ones_like(u)`` inside a traced callable (only fed to
    ``torch.autograd.grad`` as the cotangent, see :func:`autodiff._routed_autograd_grad`)."""


class _TraceCtx(autodiff._Ctx):
    """tdq.grad / u_model resolution while tracing (mirrors :class:`autodiff.JetContext`)."""

    def __init__(self, g, seg, coords):
        super().__init__(coords)
        self.g, self.seg = g, seg

    def proxy(self):
        def u_model(*args, **kw):
            s = Sym(self.g, self.g.add(("stream", self.seg, ())))
            self.register(s, (), False)
            return s
        return u_model

    def grad(self, y, x):
        info = self.lookup(y)
        var = self.var_of.get(id(x))
        if info is None or var is None:
            raise TraceError("grad() of a tensor that is not a derivative stream of u_model")
        mi = tuple(sorted(info[0] + (var,)))
        s = Sym(self.g, self.g.add(("stream", self.seg, mi)))
        self.register(s, mi, False)
        return s


def trace_callable(g, fn, seg, d_in, extra=()):
    """Trace ``fn(u_model, *extra, *coords)`` for segment slot ``seg``; returns list of Sym outputs."""
    coords = [Sym(g, g.add(("coord", seg, j))) for j in range(d_in)]
    ctx = _TraceCtx(g, seg, coords)
    with autodiff.use(ctx):
        out = fn(ctx.proxy(), *extra, *coords)
    outs = list(out) if isinstance(out, (tuple, list)) else [out]
    res = []
    for o in outs:
        if isinstance(o, Sym):
            res.append(o)
        elif isinstance(o, (list, tuple)) and len(o) == 1 and isinstance(o[0], Sym):
            res.append(o[0])
        else:
            # a constant output (e.g. u_x of a linear net) is a valid, constant residual
            res.append(Sym(g, g.add(("const", float(torch.as_tensor(o).reshape(-1)[0])))))
    return res


class Program:
    """Compiled bytecode for one segment group (one thread per instance)."""

    def __init__(self):
        self.code = []        # [op, dst, a, b]
        self.consts = []
        self.outputs = []     # (f_reg, w_reg, term_id, c)
        self.stream_regs = {}  # (seg_slot, stream_index) -> reg
        self.n_regs = 0


def compile_graph(g, outputs, stream_index, n_streams, val_ids, lam_ids, scal_ids):
    """Topologically ordered SSA bytecode for the nodes reachable from ``outputs``."""
    need = set()
    stack = [o[0] for o in outputs] + [o[1] for o in outputs]
    while stack:
        i = stack.pop()
        if i in need:
            continue
        need.add(i)
        k = g.nodes[i]
        if k[0] in ("add", "sub", "mul", "div"):
            stack += [k[1], k[2]]
        elif k[0] in ("powi", "powf") or k[0] in UNARY:
            stack.append(k[1])
    order = sorted(need)  # node ids are created in dependency order
    if len(order) > MAX_REGS:
        raise TraceError(f"fused loss program needs {len(order)} registers (> {MAX_REGS})")
    P = Program()
    reg = {}
    for i in order:
        k = g.nodes[i]
        r = len(reg)
        reg[i] = r
        kind = k[0]
        if kind == "stream":
            _, seg, mi = k
            if mi not in stream_index:
                raise TraceError(f"stream {mi} not in the jet plan")
            P.code.append([OP["STREAM"], r, seg, stream_index[mi]])
            P.stream_regs[(seg, stream_index[mi])] = r
        elif kind == "coord":
            P.code.append([OP["COORD"], r, k[1], k[2]])
        elif kind == "val":
            P.code.append([OP["VAL"], r, val_ids[k[1]], 0])
        elif kind == "lam":
            P.code.append([OP["LAM"], r, lam_ids[k[1]], 0])
        elif kind == "scal":
            P.code.append([OP["SCAL"], r, scal_ids[k[1]], 0])
        elif kind == "const":
            P.consts.append(k[1])
            P.code.append([OP["CONST"], r, len(P.consts) - 1, 0])
        elif kind in ("add", "sub", "mul", "div"):
            P.code.append([OP[kind.upper()], r, reg[k[1]], reg[k[2]]])
        elif kind == "powi":
            P.code.append([OP["POWI"], r, reg[k[1]], k[2]])
        elif kind == "powf":
            P.consts.append(k[2])
            P.code.append([OP["POWF"], r, reg[k[1]], len(P.consts) - 1])
        elif kind in UNARY:
            P.code.append([OP[UNARY[kind]], r, reg[k[1]], 0])
        else:  # pragma: no cover
            raise TraceError(kind)
    P.outputs = [(reg[f], reg[w], t, c) for (f, w, t, c) in outputs]
    P.n_regs = len(reg)
    return P


class Group:
    """Instances = points of the primary segment (periodic: partner segment read at same i)."""

    def __init__(self, segs, n):
        self.segs = segs   # segment indices read by this group (slot order)
        self.n = n
        self.program = None


class FusedLoss:
    """Everything the fused kernel needs for one LossProgram."""

    def __init__(self):
        self.groups = []
        self.term_names = []
        self.val_arrays = []      # tensors (n,) per val id
        self.lam_slots = []       # lambda index (into solver lambdas) per lam id
        self.scal_slots = []      # ("lam", index) or ("extra", k) per scalar id
        self.lam_offsets = {}     # lambda index -> (lo, hi) slice read by a minibatch program
        self.n_streams = 0


def _weight(g, lam_sym, kind_g, gfun):
    if lam_sym is None:
        return Sym(g, g.add(("const", 1.0)))
    if gfun is not None:
        w = gfun(lam_sym)
        if not isinstance(w, Sym):
            raise TraceError("g(lambda) must depend on lambda")
        return w
    if kind_g == "outside":
        return lam_sym
    return lam_sym * lam_sym


def build(prog, lambdas, extras_example=None):
    """Compile a :class:`~tensordiffeq_amd.models.loss.LossProgram` into a :class:`FusedLoss`.

    Returns ``None`` if any term cannot be fused (the caller keeps the autograd loss)."""
    if prog.plan is None or prog.backend not in ("hip", "jet"):
        return None
    if prog.net.layer_sizes[-1] != 1:
        return None
    try:
        return _build(prog, lambdas)
    except Exception as e:  # any tracing problem -> keep the autograd-composed loss
        prog.reasons.append(f"loss fusion disabled: {e}")
        return None


def _build(prog, lambdas):
    fl = FusedLoss()
    # mixed programs: the main plan's rows, then the high-order rows (LossProgram.fused_streams)
    stream_index, fl.n_streams = prog.fused_streams()
    g_by_seg = {}
    gs = []
    lam_id = {}
    scal_id = {}

    def group_for(segs):
        key = tuple(segs)
        for gr, g in gs:
            if set(gr.segs) & set(segs):
                if tuple(gr.segs) != key and not set(segs) <= set(gr.segs):
                    raise TraceError("segments shared across incompatible groups")
                return gr, g
        n = prog.segments[segs[0]].n
        if any(prog.segments[s].n != n for s in segs):
            raise TraceError("grouped segments differ in length")
        gr = Group(list(segs), n)
        g = Graph()
        gr.outputs = []
        gs.append((gr, g))
        return gr, g

    def lam_sym(g, t):
        if t.lam is None:
            return None
        lam = lambdas[t.lam]
        if lam.numel() == 1:
            if ("lam", t.lam) not in scal_id:
                scal_id[("lam", t.lam)] = len(fl.scal_slots)
                fl.scal_slots.append(("lam", t.lam))
            return Sym(g, g.add(("scal", ("lam", t.lam))))
        if prog.weight_outside_sum:
            raise TraceError("outside-sum weighting with per-point weights")
        if t.lam not in lam_id:
            lam_id[t.lam] = len(fl.lam_slots)
            fl.lam_slots.append(t.lam)
        rng = getattr(t, "lam_range", None)
        if rng is not None:
            if fl.lam_offsets.get(t.lam, rng) != rng:
                raise TraceError("one lambda read through two different slices")
            fl.lam_offsets[t.lam] = rng
        return Sym(g, g.add(("lam", t.lam)))

    def val_sym(g, t, val, n):
        v = val if torch.is_tensor(val) else torch.as_tensor(val, dtype=torch.float32)
        if v.numel() == 1:
            return Sym(g, g.add(("const", float(v.reshape(()).item()))))
        vid = len(fl.val_arrays)
        fl.val_arrays.append(v.reshape(-1).to(torch.float32).contiguous())
        return Sym(g, g.add(("val", vid)))

    osum = "outside" if prog.weight_outside_sum else "inside"
    for ti, t in enumerate(prog.terms):
        fl.term_names.append(t.name)
        c_base = t.scale
        if t.kind in ("dirichlet", "ic", "data"):
            gr, g = group_for([t.seg])
            slot = gr.segs.index(t.seg)
            n = prog.segments[t.seg].n
            u = Sym(g, g.add(("stream", slot, ())))
            f = u - val_sym(g, t, t.val, n)
            w = _weight(g, lam_sym(g, t), osum, None)
            c = c_base / (t.denom if t.denom is not None else n)
            gr.outputs.append((f.i, w.i, ti, c))
        elif t.kind == "residual":
            gr, g = group_for([t.seg])
            slot = gr.segs.index(t.seg)
            n = prog.segments[t.seg].n
            key = ("res", id(t.fn), t.seg)
            if key not in g_by_seg:
                extra = tuple(_extra_syms(g, t.extra, scal_id, fl))
                g_by_seg[key] = trace_callable(g, t.fn, slot, prog.d_in, extra)
            f = g_by_seg[key][t.index]
            ls = lam_sym(g, t)
            gfun = prog.g if (ls is not None and prog.g is not None) else None
            w = _weight(g, ls, osum, gfun)
            c = c_base / (t.denom if t.denom is not None else n)
            gr.outputs.append((f.i, w.i, ti, c))
        elif t.kind == "periodic":
            for su, sl in t.pairs:
                gr, g = group_for([su, sl])
                n = prog.segments[su].n
                ou, ol = [], []
                for fn in t.fns:
                    ou += trace_callable(g, fn, gr.segs.index(su), prog.d_in)
                    ol += trace_callable(g, fn, gr.segs.index(sl), prog.d_in)
                    if prog.periodic_legacy:
                        break
                if prog.periodic_legacy:
                    ou, ol = ou[:1], ol[:1]
                for a, b in zip(ou, ol):
                    f = a - b
                    w = _weight(g, lam_sym(g, t), osum, None)
                    gr.outputs.append((f.i, w.i, ti, c_base / n))
        elif t.kind == "neumann":
            for si in t.segs:
                gr, g = group_for([si])
                n = prog.segments[si].n
                v = val_sym(g, t, t.val, n)
                for fn in t.fns:
                    for o in trace_callable(g, fn, gr.segs.index(si), prog.d_in):
                        f = v - o
                        w = _weight(g, lam_sym(g, t), osum, None)
                        gr.outputs.append((f.i, w.i, ti, c_base / n))
        else:
            raise TraceError(t.kind)
    val_ids = {i: i for i in range(len(fl.val_arrays))}
    lam_ids = {k: i for i, k in enumerate(fl.lam_slots)}
    for gr, g in gs:
        gr.program = compile_graph(g, gr.outputs, stream_index, fl.n_streams, val_ids, lam_ids, scal_id)
        gr.graph = g
        fl.groups.append(gr)
    fl.compile_ctx = (stream_index, fl.n_streams, val_ids, lam_ids, scal_id)
    return fl


def split_by_streams(fl, gr, n_lo):
    """``(P_lo, P_hi)``: the group's outputs that read only J rows ``< n_lo`` (the main plan's
    streams) and those that read only rows ``>= n_lo`` (a mixed program's high-order streams),
    each compiled on its own - a term is a sum of per-output squares, so the two programs together
    are the group's loss.  ``None`` when an output reads both kinds or one side is empty."""
    g = getattr(gr, "graph", None)
    ctx = getattr(fl, "compile_ctx", None)
    if g is None or ctx is None:
        return None
    stream_index = ctx[0]

    def rows(i):
        seen, stack, out = set(), [i], set()
        while stack:
            j = stack.pop()
            if j in seen:
                continue
            seen.add(j)
            k = g.nodes[j]
            if k[0] == "stream":
                out.add(stream_index[k[2]])
            elif k[0] in ("add", "sub", "mul", "div"):
                stack += [k[1], k[2]]
            elif k[0] in ("powi", "powf") or k[0] in UNARY:
                stack.append(k[1])
        return out

    lo, hi = [], []
    for o in gr.outputs:
        r = rows(o[0]) | rows(o[1])
        if all(x < n_lo for x in r):
            lo.append(o)
        elif all(x >= n_lo for x in r):
            hi.append(o)
        else:
            return None
    if not lo or not hi:
        return None
    P_lo, P_hi = compile_graph(g, lo, *ctx), compile_graph(g, hi, *ctx)
    # both kernels ASSIGN the per-point SA-weight gradient (dlam[a][i] = g) and run concurrently in
    # the split layout: a weight read by both programs would get only one program's adjoint (a
    # race).  The caller falls back to another layout instead.
    if _lam_ids(P_lo) & _lam_ids(P_hi):
        return None
    return P_lo, P_hi


def _lam_ids(P):
    """Per-point SA-weight slots a compiled group program loads."""
    return {a for (op, _, a, _) in P.code if op == OP["LAM"]}


def _extra_syms(g, extra, scal_id, fl):
    """DiscoveryModel passes ``(vars_list,)``: every scalar tensor becomes a scalar input."""
    out = []
    for e in extra:
        if isinstance(e, (list, tuple)):
            lst = []
            for k, v in enumerate(e):
                key = ("extra", k)
                if key not in scal_id:
                    scal_id[key] = len(fl.scal_slots)
                    fl.scal_slots.append(key)
                lst.append(Sym(g, g.add(("scal", key))))
            out.append(lst)
        else:
            raise TraceError("unsupported extra argument")
    return out


# ------------------------------------------------------------------------------------------
# reference executor (torch): the numerical definition of the fused kernel
# ------------------------------------------------------------------------------------------
def run_reference(fl, prog, J, lambdas, scalars):
    """Evaluate ``(loss_per_term, total)`` with torch autograd-able ops (same math as the kernel)."""
    losses = [None] * len(fl.term_names)
    for gr in fl.groups:
        P = gr.program
        n = gr.n
        vals = []
        for op, dst, a, b in P.code:
            if op == OP["STREAM"]:
                s = prog.segments[gr.segs[a]]
                v = J[b, s.offset:s.offset + n, 0]
            elif op == OP["COORD"]:
                s = prog.segments[gr.segs[a]]
                v = prog.X_all[s.offset:s.offset + n, b]
            elif op == OP["VAL"]:
                v = fl.val_arrays[a].to(J.device)
            elif op == OP["CONST"]:
                v = torch.full((n,), P.consts[a], device=J.device)
            elif op == OP["LAM"]:
                k = fl.lam_slots[a]
                lo, hi = fl.lam_offsets.get(k, (0, lambdas[k].shape[0]))
                v = lambdas[k].reshape(-1)[lo:hi]
            elif op == OP["SCAL"]:
                v = scalars[a].reshape(()).expand(n)
            else:
                x = vals[a]
                if op == OP["ADD"]:
                    v = x + vals[b]
                elif op == OP["SUB"]:
                    v = x - vals[b]
                elif op == OP["MUL"]:
                    v = x * vals[b]
                elif op == OP["DIV"]:
                    v = x / vals[b]
                elif op == OP["NEG"]:
                    v = -x
                elif op == OP["POWI"]:
                    v = x ** b
                elif op == OP["POWF"]:
                    v = x ** P.consts[b]
                elif op == OP["SQUARE"]:
                    v = x * x
                else:
                    v = {OP["SIN"]: torch.sin, OP["COS"]: torch.cos, OP["EXP"]: torch.exp,
                         OP["TANH"]: torch.tanh, OP["LOG"]: torch.log, OP["SQRT"]: torch.sqrt}[op](x)
            vals.append(v)
        for (fr, wr, t, c) in P.outputs:
            contrib = c * (vals[wr] * vals[fr] * vals[fr]).sum()
            losses[t] = contrib if losses[t] is None else losses[t] + contrib
    losses = [l if l is not None else torch.zeros((), device=J.device) for l in losses]
    return losses


def scalar_values(fl, lambdas, extras):
    out = []
    for kind, k in fl.scal_slots:
        if kind == "lam":
            out.append(lambdas[k].reshape(()))
        else:
            out.append(extras[0][k].reshape(()))
    return out
