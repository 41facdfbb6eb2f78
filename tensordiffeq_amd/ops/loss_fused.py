"""Host side of the fused loss kernel (``csrc/loss_fused.hip``).

Built once per :class:`~tensordiffeq_amd.models.loss.LossProgram` from its traced
:class:`~tensordiffeq_amd.fusion.FusedLoss`: bytecode, constants, outputs, the group table and a
pointer table are uploaded to device buffers; every output buffer (dJ, dlam, block partials,
losses, scalar grads) is persistent, so a captured HIP graph replays the same pointers.
"""
from __future__ import annotations

import ctypes
import math

import numpy as np
import torch

from . import _lib
from ..fusion import OP

LF_BLOCK = 128
MAX_GROUPS, MAX_SLOTS, MAX_VAL, MAX_LAM, MAX_SCAL, MAX_TERMS = 32, 2, 16, 8, 8, 32


class FusedLossOp:
    def __init__(self, fl, prog, lambdas, scalars, lam_offsets=None):
        dev = prog.device
        if len(fl.groups) > MAX_GROUPS or len(fl.val_arrays) > MAX_VAL or len(fl.lam_slots) > MAX_LAM \
                or len(fl.scal_slots) > MAX_SCAL or len(fl.term_names) > MAX_TERMS:
            raise ValueError("fused loss program exceeds kernel table limits")
        self.fl, self.prog = fl, prog
        code, consts, outs, groups = [], [], [], []
        self.group_meta = []   # (block_off, phase, n, seg_off, n_slots, loaded) per group (ops/loss_jit.py)
        spans = []
        block_off = 0
        self.max_regs = 1
        for gr in fl.groups:
            P = gr.program
            if len(gr.segs) > MAX_SLOTS:
                raise ValueError("group reads more than 2 segments")
            loaded = [0] * MAX_SLOTS
            for (slot, s) in P.stream_regs:
                loaded[slot] |= 1 << s
            offs = [prog.segments[s].offset for s in gr.segs]
            seg_off = offs + [0] * (MAX_SLOTS - len(gr.segs))
            # single-segment groups: block boundaries on absolute multiples of LF_BLOCK (LFGroup.phase)
            phase = offs[0] % LF_BLOCK if len(offs) == 1 else 0
            groups.append([len(code), len(P.code), len(consts), P.n_regs, gr.n, block_off, len(outs),
                           len(P.outputs), len(gr.segs)] + seg_off + loaded + [phase])
            self.group_meta.append((block_off, phase, gr.n, list(seg_off), len(gr.segs), list(loaded)))
            code += P.code
            consts += P.consts
            outs += P.outputs
            nb = max(1, math.ceil((gr.n + phase) / LF_BLOCK))
            for k in range(nb):  # the point span every block reads / writes (range launches)
                a, b = max(0, k * LF_BLOCK - phase), min(gr.n, (k + 1) * LF_BLOCK - phase) - 1
                if b < a:
                    spans.append((math.inf, -math.inf))
                else:
                    spans.append((min(o + a for o in offs), max(o + b for o in offs)))
            block_off += nb
            self.max_regs = max(self.max_regs, P.n_regs)
        self.n_blocks = block_off
        self.block_spans = spans
        self.n_groups = len(groups)
        self.n_terms = len(fl.term_names)
        self.n_scal = len(fl.scal_slots)
        self.code = torch.tensor(np.asarray(code, dtype=np.int32).reshape(-1, 4), device=dev)
        self.consts = torch.tensor(np.asarray(consts + [0.0], dtype=np.float32), device=dev)
        ob = np.zeros(max(1, len(outs)), dtype=[("f", "<i4"), ("w", "<i4"), ("t", "<i4"), ("c", "<f4")])
        for k, (f, w, t, c) in enumerate(outs):
            ob[k] = (f, w, t, c)
        self.outs = torch.from_numpy(ob.view(np.uint8).copy()).to(dev)
        ga = np.asarray(groups, dtype=np.int32)
        if dev.type == "cuda":
            sizes = (ctypes.c_int * 4)()
            _lib.load().tdq_loss_meta_sizes(sizes)
            if sizes[3] != 4 * ga.shape[1]:
                raise RuntimeError(f"LFGroup is {sizes[3]} bytes in libtdq_hip.so, {4 * ga.shape[1]} here; rebuild")
        self.groups = torch.tensor(ga, device=dev)
        # persistent inputs / outputs
        self.vals = [v.to(dev).contiguous() for v in fl.val_arrays]
        lam_offsets = lam_offsets or {}
        self.lams = lambdas
        self.dlam = []
        for k in fl.lam_slots:
            lo, hi = lam_offsets.get(k, (0, lambdas[k].shape[0]))
            self.dlam.append(torch.zeros(hi - lo, device=dev))
        self.scalars = scalars
        ptrs = np.zeros(MAX_VAL + 3 * MAX_LAM + MAX_SCAL, dtype=np.int64)
        ptrs[MAX_VAL + 3 * MAX_LAM:] = 0
        for i, v in enumerate(self.vals):
            ptrs[i] = v.data_ptr()
        for i, k in enumerate(fl.lam_slots):
            lo = lam_offsets.get(k, (0, 0))[0]
            ptrs[MAX_VAL + i] = lambdas[k].data_ptr() + 4 * lo
            ptrs[MAX_VAL + MAX_LAM + i] = self.dlam[i].data_ptr()
        for i, s in enumerate(scalars):
            ptrs[MAX_VAL + 2 * MAX_LAM + i] = s.data_ptr()
        # layout of LFPtrs: val[16], lam[8], dlam[8], scal[8]
        self.ptrs = torch.from_numpy(ptrs[:MAX_VAL + 2 * MAX_LAM + MAX_SCAL].copy()).to(dev)
        N = prog.X_all.shape[0]
        self.N = N
        self.dJ = torch.zeros((fl.n_streams, N, 1), device=dev)
        self.partials = torch.zeros(self.n_blocks * (self.n_terms + self.n_scal), device=dev)
        self.losses = torch.zeros(self.n_terms, device=dev)
        self.total = torch.zeros((), device=dev)
        self.dscal = torch.zeros(max(1, self.n_scal), device=dev)
        # the program compiled to a specialized kernel (hipRTC), or None: the interpreter
        from . import loss_jit
        self.jit = loss_jit.compile_for(self)

    @property
    def engine(self):
        return "jit" if self.jit is not None else "interpreter"

    def __call__(self, J, with_total=True, reduce=True):
        """Run the program on jets ``J``.  ``with_total=False`` skips the total-loss launch (the Adam
        step's bookkeeping kernel sums the terms instead; ``total`` is then stale until it runs).
        ``reduce=False``: only the loss kernel (dJ, SA-weight gradients, block partials); the
        per-term losses and scalar gradients are reduced by the fused step tail
        (``jet_hip.step_tail`` / ``jet_hip.dp_tail_a``)."""
        lib = _lib.load()
        if self.jit is not None:
            st = _lib.stream_ptr(J.device)
            self.jit.launch(J, self.prog.X_all, self.dJ, self.partials, self.ptrs, 0, self.n_blocks, st)
            if reduce:
                rc = lib.tdq_loss_reduce_partials(_lib.ptr(self.partials), self.n_blocks, self.n_terms, self.n_scal,
                                                  _lib.ptr(self.losses), _lib.ptr(self.total), _lib.ptr(self.dscal),
                                                  int(bool(with_total)), st)
                _lib.check(rc, "tdq_loss_reduce_partials")
            return self.total, self.losses, self.dJ, self.dlam, self.dscal
        rc = lib.tdq_loss_fused(_lib.ptr(self.code), _lib.ptr(self.consts), _lib.ptr(self.outs),
                                _lib.ptr(self.groups), _lib.ptr(self.ptrs), self.n_groups, self.n_terms,
                                self.n_scal, self.fl.n_streams, self.prog.d_in, self.N, _lib.ptr(J),
                                _lib.ptr(self.prog.X_all), _lib.ptr(self.dJ), _lib.ptr(self.partials),
                                self.n_blocks, self.max_regs, _lib.ptr(self.losses), _lib.ptr(self.total),
                                _lib.ptr(self.dscal), int(bool(with_total)), int(bool(reduce)),
                                _lib.stream_ptr(J.device))
        _lib.check(rc, "tdq_loss_fused")
        return self.total, self.losses, self.dJ, self.dlam, self.dscal

    def split_block(self, a):
        """Block index ``b`` such that blocks ``[0, b)`` touch only points ``< a`` and blocks
        ``[b, n_blocks)`` only points ``>= a`` (so the two ranges can run as separate launches
        next to the jet kernels of their point ranges), or ``None``."""
        b = 0
        while b < self.n_blocks and self.block_spans[b][1] < a:
            b += 1
        if b == 0 or b == self.n_blocks:
            return None
        if any(lo < a for lo, _ in self.block_spans[b:]):
            return None
        return b

    def run_range(self, J, blk0, nblk):
        """Blocks ``[blk0, blk0 + nblk)`` only (dJ / dlam / block partials of their points; the
        fused step tail reduces the partials), on the current stream."""
        lib = _lib.load()
        if self.jit is not None:
            self.jit.launch(J, self.prog.X_all, self.dJ, self.partials, self.ptrs, blk0, nblk,
                            _lib.stream_ptr(J.device))
            return
        rc = lib.tdq_loss_fused_range(_lib.ptr(self.code), _lib.ptr(self.consts), _lib.ptr(self.outs),
                                      _lib.ptr(self.groups), _lib.ptr(self.ptrs), self.n_groups, self.n_terms,
                                      self.n_scal, self.fl.n_streams, self.prog.d_in, self.N, _lib.ptr(J),
                                      _lib.ptr(self.prog.X_all), _lib.ptr(self.dJ), _lib.ptr(self.partials),
                                      self.n_blocks, int(blk0), int(nblk), self.max_regs,
                                      _lib.stream_ptr(J.device))
        _lib.check(rc, "tdq_loss_fused_range")

