"""Layer-wise jet engine for hidden widths beyond the fused kernels (``csrc/jet_layered.hip``).

The fused jet kernels keep all derivative streams of a 16-point tile in registers through the
whole layer stack, which bounds the hidden width at 128.  The reference accepts any layer list
(``tensordiffeq/networks.py:10-20``), so wider networks run one layer at a time:

* the S derivative streams of a layer are stacked into one ``[S*N, W]`` matrix, so every weight
  multiplication of a layer - forward ``Z = H K``, backward ``HB = ZB K^T`` and the weight gradient
  ``dK = H^T ZB`` (reduction over all streams and points at once) - is ONE GEMM in the requested
  precision family: fp32, bf16 (operands rounded once, fp32 accumulation) or bf16x3 (hi/lo split:
  hi*hi + hi*lo + lo*hi).  On the GPU these are the hand-written MFMA kernels of
  ``csrc/lay_gemm.hip`` (``TDQ_LAY_GEMM=0``: the library GEMMs through ``torch.mm``, the A/B
  reference);
* the bias, the tanh jet (value, first-, second-order streams) and its adjoint (``csrc/lay_jet.h``)
  run in the EPILOGUE of the hidden layers' NN GEMMs (``tdq_lay_nnj``: a GEMM tile holds all S
  streams of its points, so the jet runs on the accumulators); in the bf16 families the layer's
  output leaves the kernel only as the next GEMMs' bf16 operands, whose hi + lo sum is also the
  saved post-activation of the adjoint (fp32: one fp32 plane) - no Z / HB round trips through HBM.
  The input layer is one ``X K0`` + jet kernel, the last hidden layer's adjoint forms ``dJ Ko^T``
  in-kernel, and the input layer's gradient leaves as tile partials.  The library path
  (``TDQ_LAY_GEMM=0``), ``TDQ_LAY_FUSED=0`` and CPU use the standalone memory-bound epilogue pass
  (``tdq_layered_epi``) between plain GEMMs.

Orders <= 2 (like the fused kernels).  On CPU the same engine runs with torch epilogues (the
numerics oracle of the HIP pass, tests/test_layered_jet.py).  Same contract as
:func:`.jet_hip.forward_raw` / :func:`.jet_hip.backward_raw`: ``J`` is ``(S, N, d_out)``.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib


def _spec(plan):
    from .jet_hip import stream_spec
    return stream_spec(plan)


def _epi_fwd_torch(Z, bias, spec):
    """In place Z -> H (torch mirror of ``layered_fwd_kernel``)."""
    S = Z.shape[0]
    z = Z.clone()
    h = torch.tanh(z[0] + bias)
    s1 = 1 - h * h
    Z[0] = h
    for s in range(1, S):
        ty, a, b = spec[3 * s:3 * s + 3]
        Z[s] = s1 * z[s] if ty == 1 else s1 * (z[s] - 2 * h * z[a] * z[b])
    return Z


def _epi_bwd_torch(HB, H, spec):
    """In place HB -> ZB (torch mirror of ``layered_bwd_kernel``)."""
    S = HB.shape[0]
    hb = HB.clone()
    h0 = H[0]
    s1 = 1 - h0 * h0
    acc0 = s1 * hb[0]
    zb = [None] + [s1 * hb[s] for s in range(1, S)]
    for s in range(1, S):
        acc0 = acc0 - 2 * h0 * H[s] * hb[s]
    for s in range(1, S):
        ty, a, b = spec[3 * s:3 * s + 3]
        if ty != 2:
            continue
        acc0 = acc0 - 2 * H[a] * H[b] * hb[s]
        zb[a] = zb[a] - 2 * h0 * H[b] * hb[s]
        zb[b] = zb[b] - 2 * h0 * H[a] * hb[s]
    HB[0] = acc0
    for s in range(1, S):
        HB[s] = zb[s]
    return HB


class _Op:
    """A GEMM operand in the engine's precision: fp32 as is; ``bf16`` one rounded copy; ``bf16x3``
    a (hi, lo) split (products hi*hi + hi*lo + lo*hi, fp32 accumulation - the fused kernels'
    precision families).  Built once per activation / adjoint and reused by every GEMM reading it."""

    def __init__(self, x, prec):
        self.prec = prec
        if prec == "fp32" or not x.is_cuda:
            self.f = x
        else:
            self.h = x.to(torch.bfloat16)
            if prec == "bf16x3":
                self.l = (x - self.h.float()).to(torch.bfloat16)

    @classmethod
    def parts(cls, prec, h, l=None):
        """An operand whose bf16 hi (/ lo) copies were written by the epilogue pass itself."""
        o = cls.__new__(cls)
        o.prec, o.h = prec, h
        if l is not None:
            o.l = l
        return o

    def t(self):
        o = _Op.__new__(_Op)
        o.prec = self.prec
        for k in ("f", "h", "l"):
            if hasattr(self, k):
                setattr(o, k, getattr(self, k).t())
        return o


_PREC = {"bf16": 0, "bf16x3": 1, "fp32": 2}


def _hip_gemm():
    """The hand-written MFMA GEMMs (csrc/lay_gemm.hip) serve CUDA operands unless
    ``TDQ_LAY_GEMM=0`` (the library GEMMs, kept as the A/B reference)."""
    import os
    return os.environ.get("TDQ_LAY_GEMM", "1") != "0" and _lib.available()


def _planes(o):
    """(hi, lo) device planes of an operand in its precision (fp32: the tensor itself)."""
    if hasattr(o, "f"):
        return o.f, None
    return o.h, getattr(o, "l", None)


def _colsum(src, R, M, out, lds=None, W=None, sj=None, sf=1, bias=None, nbias=0):
    """``out`` element m = sum over the R rows of ``src`` (row stride ``lds``, default M) of column
    m, at ``out``'s storage offset (m // W) * sj + (m % W) * sf (defaults: contiguous) - the
    fixed-order HIP column sum (csrc/lay_reduce.hip ``tdq_colsum``) in place of ``torch.sum``;
    ``bias`` [bdim] is added to the first ``nbias`` elements."""
    lib = _lib.load(required=True)
    W = M if W is None else W
    sj = W if sj is None else sj
    nw = int(lib.tdq_colsum_work(int(R), int(M)))
    work = torch.empty(max(nw, 1), dtype=torch.float32, device=src.device) if nw > 0 else None
    _lib.check(lib.tdq_colsum(_lib.ptr(src), int(M if lds is None else lds), int(R), int(M), _lib.ptr(out), int(W),
                              int(sj), int(sf), _lib.ptr(bias), int(nbias),
                              int(bias.numel()) if bias is not None else 1, _lib.ptr(work),
                              _lib.stream_ptr(src.device)), "tdq_colsum")
    return out


def _bplanes(bt, prec):
    """The :class:`_Op` of an NN GEMM's B^T operand [Nout, K] from fp32 weights (a view of a
    contiguous tensor or its transpose): bf16 hi (/ lo) planes in one launch
    (csrc/lay_reduce.hip ``tdq_lay_bplanes``), not a transpose copy + casts."""
    if bt.is_contiguous():
        src, tr = bt, 0
    elif bt.t().is_contiguous():
        src, tr = bt.t(), 1
    else:
        return _Op(bt.contiguous(), prec)
    h = torch.empty(bt.shape, dtype=torch.bfloat16, device=bt.device)
    l = torch.empty_like(h) if prec == "bf16x3" else None
    lib = _lib.load(required=True)
    _lib.check(lib.tdq_lay_bplanes(_lib.ptr(src), src.shape[0], src.shape[1], tr, _lib.ptr(h), _lib.ptr(l),
                                   _lib.stream_ptr(bt.device)), "tdq_lay_bplanes")
    return _Op.parts(prec, h, l)


def _mm_w(a, w, prec, out=None):
    """a @ w for an activation operand ``a`` [M, K] (:class:`_Op`) and fp32 weights ``w`` [K, N]
    (the weights' transposed operand ``[N, K]`` is formed here - W x W, small)."""
    return _mm_bt(a, w.t().contiguous(), prec, out)


def _mm_bt(a, bt, prec, out=None):
    """a @ bt^T with ``bt`` [N, K] fp32: the hand-written NN GEMM on CUDA, else the library."""
    if a.prec != prec:
        raise ValueError("operand precision mismatch")
    x = a.f if hasattr(a, "f") else a.h
    if x.is_cuda and _hip_gemm():
        bo = _Op(bt, prec) if prec != "fp32" else None
        ah, al = _planes(a)
        bh, bl = (bt, None) if bo is None else _planes(bo)
        M, K = ah.shape
        N = bh.shape[0]
        c = out if out is not None else torch.empty((M, N), dtype=torch.float32, device=x.device)
        if not (c.is_contiguous() and ah.is_contiguous() and bh.is_contiguous()):
            raise ValueError("GEMM operands must be contiguous")
        lib = _lib.load(required=True)
        rc = lib.tdq_lay_nn(_PREC[prec], _lib.ptr(ah), _lib.ptr(al), K, _lib.ptr(bh), _lib.ptr(bl), K,
                            _lib.ptr(c), N, M, N, K, _lib.stream_ptr(x.device))
        _lib.check(rc, "tdq_lay_nn")
        return c
    return _mm(a, _Op(bt.t(), prec), out)


def _mm(a, b, out=None):
    """a @ b for two :class:`_Op` of the same precision (library GEMMs, fp32 output)."""
    if hasattr(a, "f"):
        return torch.mm(a.f, b.f, out=out)
    f32 = torch.float32
    r = torch.mm(a.h, b.h, out_dtype=f32)
    if a.prec == "bf16x3":
        r += torch.mm(a.h, b.l, out_dtype=f32)
        r += torch.mm(a.l, b.h, out_dtype=f32)
    if out is not None:
        out.copy_(r)
        return out
    return r


def _mm_tn(a, b, out):
    """out = a^T b for :class:`_Op` a [L, M], b [L, N] with a long reduction L = S*N (the weight
    gradient): as ONE library GEMM its M x N = W x W output is only a few tiles, so a handful of CUs
    did all the work (bf16 ~50 TF/s, profiles/r3_ag_*).  The reduction is split into C chunks - the
    hand-written TN GEMM's grid z on CUDA (csrc/lay_gemm.hip), else one batched library GEMM
    ([C, M, L/C] x [C, L/C, N]) - and the C partial products summed in fixed order."""
    x = a.f if hasattr(a, "f") else a.h
    if x.is_cuda and _hip_gemm():
        ah, al = _planes(a)
        bh, bl = _planes(b)
        L, Ma = ah.shape
        Nb = bh.shape[1]
        tiles = -(-Ma // 128) * -(-Nb // 128)
        want = max(1, min(-(-1024 // tiles), -(-L // 256)))   # >= ~1024 workgroups, >= 256 rows each
        rows = (-(-L // want) + 31) // 32 * 32                # a multiple of 32 rows per chunk
        nch = -(-L // rows)
        part = torch.empty((nch, Ma, Nb), dtype=torch.float32, device=x.device)
        lib = _lib.load(required=True)
        rc = lib.tdq_lay_tn(_PREC[a.prec], _lib.ptr(ah.contiguous()), _lib.ptr(al), Ma, _lib.ptr(bh.contiguous()),
                            _lib.ptr(bl), Nb, _lib.ptr(part), L, Ma, Nb, rows, _lib.stream_ptr(x.device))
        _lib.check(rc, "tdq_lay_tn")
        return _colsum(part, nch, Ma * Nb, out, W=Nb, sj=out.stride(0), sf=out.stride(1))
    L = x.shape[0]
    C = 64 if L >= 64 * 1024 else max(1, L // 1024)
    L0 = L - L % C

    def chunks(x):
        return x[:L0].view(C, L0 // C, x.shape[1])

    def bmm(x, y):
        if x.dtype != torch.bfloat16:
            return torch.bmm(chunks(x).transpose(1, 2), chunks(y))
        return torch.bmm(chunks(x).transpose(1, 2), chunks(y), out_dtype=torch.float32)

    pairs = [(a.f, b.f)] if hasattr(a, "f") else [(a.h, b.h)] + ([(a.h, b.l), (a.l, b.h)] if a.prec == "bf16x3" else [])
    r = None
    for x, y in pairs:
        p = bmm(x, y).sum(0)
        if L0 < L:
            xt, yt = x[L0:], y[L0:]
            p += (torch.mm(xt.t(), yt) if x.dtype != torch.bfloat16 else
                  torch.mm(xt.t(), yt, out_dtype=torch.float32))
        r = p if r is None else r + p
    out.copy_(r)
    return out


def _fused(X, ws, precision):
    """The GEMM-epilogue path (the layer jet inside the hand-written kernels, bf16 families)."""
    import os
    return (X.is_cuda and precision in ("bf16", "bf16x3", "fp32") and _hip_gemm() and X.shape[1] <= 8
            and os.environ.get("TDQ_LAY_FUSED", "1") != "0" and all(K.shape[1] % 4 == 0 for K, _ in ws[:-1]))


EPI_FWD, EPI_BWD, EPI_BWD0 = 0, 1, 2   # csrc/lay_gemm.hip lay_epilogue modes


def _spec_c(spec):
    return (ctypes.c_int * len(spec))(*spec)


def _hl(H):
    """(hi, lo) device planes of a saved activation: a bf16 pair, or one fp32 plane (fp32 engine)."""
    if H is None:
        return None, None
    return H if isinstance(H, tuple) else (H, None)


def _nnj(mode, prec, spec, S, N, a, bt, bias=None, H=None, part=None, X=None, ko=None, jpart=None):
    """One NN GEMM with the layer jet in its epilogue (csrc/lay_gemm.hip ``lay_nnj_kernel``): ``a``
    the :class:`_Op` of the layer input planes [S*N, K], ``bt`` the fp32 B^T [Nout, K].  Returns the
    (hi, lo) bf16 output planes: EPI_FWD the layer's post-activations (lo always - it is the saved
    activation's residual), EPI_BWD its ZB (lo in bf16x3 only; ``part`` the bias partials),
    EPI_BWD0 nothing (``part`` the input layer's gradient partials, ``X`` its coordinates).  fp32:
    one fp32 output plane as ``(plane, None)``, ``H`` the fp32 plane.  EPI_FWD of the last hidden
    layer may also take the output layer (``ko`` [Nout, d_out], ``jpart`` [ceil(Nout / 64), S, N,
    d_out]): J's partial dots per 64-column group come out of the same epilogue."""
    ah, al = _planes(a)
    bo = _bplanes(bt, prec) if prec != "fp32" else None
    bh, bl = _planes(bo) if bo is not None else (bt.contiguous(), None)
    Nout, K = bt.shape
    dev = ah.device
    oh = ol = None
    if mode != EPI_BWD0:
        oh = torch.empty((S * N, Nout), dtype=torch.float32 if prec == "fp32" else torch.bfloat16, device=dev)
        if prec != "fp32" and (mode == EPI_FWD or prec == "bf16x3"):
            ol = torch.empty_like(oh)
    hh, hl = _hl(H)
    lib = _lib.load(required=True)
    rc = lib.tdq_lay_nnj(_PREC[prec], mode, S, _spec_c(spec), _lib.ptr(ah), _lib.ptr(al), _lib.ptr(bh), _lib.ptr(bl),
                         N, K, Nout, _lib.ptr(bias), _lib.ptr(hh), _lib.ptr(hl), _lib.ptr(oh), _lib.ptr(ol),
                         _lib.ptr(part), _lib.ptr(X), 0 if X is None else X.shape[1], _lib.ptr(ko), _lib.ptr(jpart),
                         0 if ko is None else ko.shape[1], _lib.stream_ptr(dev))
    _lib.check(rc, "tdq_lay_nnj")
    return oh, ol


def _parts(S, N, W, q, dev):
    """Per-tile partials of a jet epilogue: one row per tile row (128 // S points) x q x W."""
    return torch.empty((-(-N // (128 // S)), q, W), dtype=torch.float32, device=dev)


def _xtz(Xm, out, Z=None, H=None, rows=32):
    """``out[f][j] = sum_n X[n][j] Z[n][f]`` (``out`` [W, d], may be a transposed view) for fp32
    ``Xm`` [R, d] and Z [R, W] (fp32, or the (hi, lo) bf16 planes ``H``): chunked partials of the
    FMA kernel (csrc/lay_gemm.hip ``lay_xtz_kernel``, <= 8 columns per launch), fixed-order sum."""
    lib = _lib.load(required=True)
    R = Xm.shape[0]
    W = out.shape[0]
    zh, zl = H if H is not None else (None, None)
    for j0 in range(0, Xm.shape[1], 8):
        xj = Xm[:, j0:j0 + 8].contiguous()
        part = torch.empty((-(-R // rows), xj.shape[1], W), dtype=torch.float32, device=Xm.device)
        _lib.check(lib.tdq_lay_xtz2(_lib.ptr(xj), xj.shape[1], _lib.ptr(Z), _lib.ptr(zh), _lib.ptr(zl), R, W,
                                    _lib.ptr(part), rows, _lib.stream_ptr(Xm.device)), "tdq_lay_xtz2")
        # part [rows, nj, W] summed over rows: element (j, f) -> out[f][j0 + j]
        _colsum(part, part.shape[0], xj.shape[1] * W, out[:, j0:], W=W, sj=out.stride(1), sf=out.stride(0))
    return out


def _epi(fwd, A, B, bias, spec, prec="fp32", keep_lo=False, H=None):
    """The standalone epilogue pass in place on A; returns ``(A, op)`` with ``op`` the :class:`_Op`
    of the result viewed ``[S*N, W]`` - in the bf16 families its hi (/ lo) copies are written by
    the same pass instead of a separate conversion (``keep_lo``: the lo plane in bf16 too, the
    post-activation residual of the GEMM-epilogue path; then ``op.l_saved`` holds it).  Backward
    with ``B=None``: the post-activations come as the (hi, lo) bf16 planes ``H``."""
    S, N, W = A.shape
    if A.is_cuda:
        lib = _lib.load(required=True)
        c = (ctypes.c_int * len(spec))(*spec)
        hi = lo = None
        if prec in ("bf16", "bf16x3"):
            hi = torch.empty((S * N, W), dtype=torch.bfloat16, device=A.device)
            if prec == "bf16x3" or keep_lo:
                lo = torch.empty_like(hi)
        hh, hl = H if H is not None else (None, None)
        rc = lib.tdq_layered_epi(1 if fwd else 0, _lib.ptr(A), _lib.ptr(B), _lib.ptr(bias), N, W, S, c,
                                 _lib.ptr(hi), _lib.ptr(lo), _lib.ptr(hh), _lib.ptr(hl), _lib.stream_ptr(A.device))
        _lib.check(rc, "tdq_layered_epi")
        if hi is None:
            return A, _Op(A.view(S * N, W), prec)
        op = _Op.parts(prec, hi, lo if prec == "bf16x3" else None)
        op.l_saved = lo
        return A, op
    if H is not None:
        B = (H[0].float() + H[1].float()).view(S, N, W)
    A = _epi_fwd_torch(A, bias, spec) if fwd else _epi_bwd_torch(A, B, spec)
    return A, _Op(A.view(S * N, W), prec)


@torch.no_grad()
def forward_raw(X, P, net, plan, precision="fp32"):
    """``(J, saved)``; ``saved`` feeds :func:`backward_raw`.  ``precision`` of the hidden and output
    GEMMs: ``fp32``, ``bf16`` or ``bf16x3`` (the input layer is exact fp32 in every mode)."""
    spec = _spec(plan)
    ws = net.weights(P)
    S, N = plan.S, X.shape[0]
    fused = _fused(X, ws, precision)
    K0, b0 = ws[0]
    W0 = K0.shape[1]
    if fused:
        # input layer: X K0 (d_in exact fp32 FMAs) + jet in one pass, the hidden layers' NN GEMMs with
        # the jet in their epilogues; activations only as (hi, lo) bf16 planes
        f32 = precision == "fp32"
        hi = torch.empty((S * N, W0), dtype=torch.float32 if f32 else torch.bfloat16, device=X.device)
        lo = None if f32 else torch.empty_like(hi)
        lib = _lib.load(required=True)
        _lib.check(lib.tdq_lay_in_fwd(int(f32), S, _spec_c(spec), _lib.ptr(X), X.shape[1], _lib.ptr(K0.contiguous()),
                                      _lib.ptr(b0.contiguous()), N, W0, _lib.ptr(hi), _lib.ptr(lo),
                                      _lib.stream_ptr(X.device)), "tdq_lay_in_fwd")

        def saved(hi, lo):   # (saved activation, GEMM operand)
            if f32:
                return hi, _Op(hi, "fp32")
            return (hi, lo), _Op.parts(precision, hi, lo if precision == "bf16x3" else None)

        h, o = saved(hi, lo)
        Hs, Ho = [h], [o]
        Ko, bo = ws[-1]
        d_out = Ko.shape[1]
        jpart = None
        for i, (K, b) in enumerate(ws[1:-1]):
            kw = {}
            if i == len(ws) - 3 and d_out <= 4:   # the last hidden layer also forms J = H Ko
                jpart = torch.empty((-(-K.shape[1] // 64), S, N, d_out), dtype=torch.float32, device=X.device)
                kw = {"ko": Ko.contiguous(), "jpart": jpart}
            h, o = saved(*_nnj(EPI_FWD, precision, spec, S, N, Ho[-1], K.t(), bias=b, **kw))
            Hs.append(h)
            Ho.append(o)
        if jpart is not None:   # J = the 64-column partials summed, + bo on the value stream
            J = torch.empty((S, N, d_out), dtype=torch.float32, device=X.device)
            _colsum(jpart, jpart.shape[0], S * N * d_out, J, bias=bo, nbias=N * d_out)
        else:
            J = _mm_w(Ho[-1], Ko, precision).view(S, N, d_out)
            J[0] += bo
        return J, ("layered", X, P, net, spec, Hs, Ho, precision, fused)
    Z = torch.zeros((S, N, W0), dtype=P.dtype, device=X.device)
    if X.is_cuda:   # layer 0: the input is exact fp32, d_in <= 8 columns - FMAs, not a GEMM
        torch.mul(X[:, :1], K0[0], out=Z[0])
        for j in range(1, X.shape[1]):
            Z[0].addcmul_(X[:, j:j + 1], K0[j])
    else:
        torch.mm(X, K0, out=Z[0])
    for s in range(1, S):
        if spec[3 * s] == 1:
            Z[s].copy_(K0[spec[3 * s + 1]].expand(N, W0))
    H, op = _epi(True, Z, None, b0, spec, precision)
    Hs, Ho = [H], [op]                               # saved activations and their GEMM operands
    for K, b in ws[1:-1]:
        Z = _mm_w(Ho[-1], K, precision).view(S, N, K.shape[1])
        H, op = _epi(True, Z, None, b, spec, precision)
        Hs.append(H)
        Ho.append(op)
    Ko, bo = ws[-1]
    J = _mm_w(Ho[-1], Ko, precision).view(S, N, Ko.shape[1])
    J[0] += bo
    return J, ("layered", X, P, net, spec, Hs, Ho, precision, fused)


@torch.no_grad()
def backward_raw(saved, dJ, grad=None):
    """Flat parameter gradient of ``<dJ, J>`` (Keras layer order, like the fused kernels)."""
    _, X, P, net, spec, Hs, Ho, prec, fused = saved
    if grad is None:
        grad = torch.empty_like(P)
    gw = net.weights(grad)
    ws = net.weights(P)
    S, N = dJ.shape[0], dJ.shape[1]
    dJ = dJ.contiguous()
    Ko, _ = ws[-1]
    dJo = None
    last = len(ws) - 2
    if fused and dJ.shape[2] <= 64:   # dKo = H^T dJ, a few columns: FMA partials on exact dJ, H = hi + lo
        if prec == "fp32":
            _xtz(dJ.view(S * N, dJ.shape[2]), gw[-1][0], Z=Hs[last], rows=64)
        else:
            _xtz(dJ.view(S * N, dJ.shape[2]), gw[-1][0], H=Hs[last], rows=64)
    else:
        dJo = _Op(dJ.view(S * N, dJ.shape[2]), prec)
        _mm_tn(Ho[-1], dJo, gw[-1][0])
    if dJ.is_cuda and _hip_gemm():
        _colsum(dJ, N, dJ.shape[2], gw[-1][1])   # dJ[0] [N, d_out] summed over the points
    else:
        torch.sum(dJ[0], dim=0, out=gw[-1][1])
    HB = None
    if not fused or dJ.shape[2] > 4:   # (the fused path forms HB = dJ Ko^T inside lay_out_bwd_kernel)
        if dJ.shape[2] == 1:  # an outer product: a K = 1 GEMM ran 10x slower than this broadcast
            HB = (dJ.view(S * N, 1) * Ko.view(1, -1)).view(S, N, Ko.shape[0])
        else:
            dJo = dJo if dJo is not None else _Op(dJ.view(S * N, dJ.shape[2]), prec)
            HB = _mm_bt(dJo, Ko, prec).view(S, N, Ko.shape[0])
    part0 = ZB0 = None
    if fused:
        d_in, d_out = X.shape[1], dJ.shape[2]
        lib = _lib.load(required=True)
        W = Ko.shape[0]
        ZBo = db = None
        f32 = prec == "fp32"
        if d_out <= 4:   # the last hidden layer's adjoint with HB = dJ Ko^T formed in the kernel
            mode = EPI_BWD if last > 0 else EPI_BWD0
            oh = ol = None
            if last > 0:
                db = _parts(S, N, W, 1, X.device)
                oh = torch.empty((S * N, W), dtype=torch.float32 if f32 else torch.bfloat16, device=X.device)
                ol = torch.empty_like(oh) if prec == "bf16x3" else None
            else:
                part0 = db = _parts(S, N, W, S + d_in, X.device)
            hh, hl = _hl(Hs[last])
            _lib.check(lib.tdq_lay_out_bwd(int(f32), mode, S, _spec_c(spec), _lib.ptr(dJ), d_out,
                                           _lib.ptr(Ko.contiguous()), _lib.ptr(hh), _lib.ptr(hl), N, W, _lib.ptr(oh),
                                           _lib.ptr(ol), _lib.ptr(db), _lib.ptr(X if last == 0 else None),
                                           d_in, _lib.stream_ptr(X.device)), "tdq_lay_out_bwd")
            if last > 0:
                ZBo = _Op(oh, "fp32") if f32 else _Op.parts(prec, oh, ol)
        elif f32:        # (wide outputs: HB from the NN GEMM, then the standalone pass)
            ZB, ZBo = _epi(False, HB, Hs[last], None, spec, "fp32")
            db = ZB[0].unsqueeze(0)
            if last == 0:
                ZB0 = ZB
        else:
            ZB, ZBo = _epi(False, HB, None, None, spec, prec if last > 0 else "fp32", H=Hs[last])
            db = ZB[0].unsqueeze(0)
            if last == 0:
                ZB0 = ZB
        for i in range(last, 0, -1):
            K, _ = ws[i]
            _mm_tn(Ho[i - 1], ZBo, gw[i][0])
            dbr = db.reshape(-1, db.shape[-1])
            _colsum(dbr, dbr.shape[0], dbr.shape[1], gw[i][1], lds=dbr.stride(0))
            # HB_{i-1} = ZB_i K_i^T with layer i-1's adjoint jet in the GEMM epilogue (K is the B^T
            # operand); the input layer's comes out as gradient partials only
            W = K.shape[0]
            if i - 1 > 0:
                db = _parts(S, N, W, 1, X.device)
                hi, lo = _nnj(EPI_BWD, prec, spec, S, N, ZBo, K, H=Hs[i - 1], part=db)
                ZBo = _Op(hi, "fp32") if f32 else _Op.parts(prec, hi, lo)
            else:
                part0 = _parts(S, N, W, S + d_in, X.device)
                _nnj(EPI_BWD0, prec, spec, S, N, ZBo, K, H=Hs[0], part=part0, X=X)
    dK0, gb0 = gw[0]
    if part0 is not None:
        # [S + d_in, W0]: stream sums, then X^T zb -> dK0 (+ first-order streams), b0
        tot = torch.empty(part0.shape[1:], dtype=torch.float32, device=part0.device)
        _colsum(part0, part0.shape[0], tot.numel(), tot)
        lib = _lib.load(required=True)
        _lib.check(lib.tdq_lay_l0grad(_lib.ptr(tot), S, X.shape[1], _spec_c(spec), tot.shape[1], _lib.ptr(dK0),
                                      _lib.ptr(gb0), _lib.stream_ptr(tot.device)), "tdq_lay_l0grad")
        return grad
    if ZB0 is None:
        for i in range(last, 0, -1):
            K, _ = ws[i]
            ZB, ZBo = _epi(False, HB, Hs[i], None, spec, prec)
            _mm_tn(Ho[i - 1], ZBo, gw[i][0])
            torch.sum(ZB[0], dim=0, out=gw[i][1])
            # HB = ZB K^T: K itself is the transposed operand [W_in, W_out] of the NN GEMM (library path:
            # K^T materialized - its transposed-B kernels ran ~4x slower, profiles/r3_ag_*)
            HB = _mm_bt(ZBo, K, prec).view(S, N, K.shape[0])
        ZB0, _ = _epi(False, HB, Hs[0], None, spec)
    if X.is_cuda and _hip_gemm():   # X^T ZB0: d_in rows of exact fp32 - chunked FMA partials
        _xtz(X, dK0.t(), Z=ZB0[0].contiguous())
    else:
        torch.mm(X.t(), ZB0[0], out=dK0)
    for s in range(1, S):
        if spec[3 * s] == 1:
            dK0[spec[3 * s + 1]] += ZB0[s].sum(dim=0)
    torch.sum(ZB0[0], dim=0, out=gb0)
    return grad
