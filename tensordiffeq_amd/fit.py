"""Training engines (reference tensordiffeq/fit.py: ``fit`` 17-102, ``train_op_inner`` 125-147,
``fit_dist`` 150-224, ``lbfgs_train`` 107-122).

:class:`AdamEngine` - one optimizer step is: loss + grads (jet kernels / autograd), the DP
bucket all-reduce, device-side best-model tracking (before the update, so the snapshot is the
weights that produced the loss - B8), one Keras-Adam update of theta and one Adam *ascent* update
of the self-adaptive weights (fused HIP kernel on GPU), and a device-side loss-history write.
Nothing in the step reads back to the host, so on a GPU the whole step is captured once into a
HIP graph and replayed (reference: a ``tf.function`` step plus a host sync every epoch,
fit.py:41-55).  Under DP the collective sits between two captured graphs.

:class:`LossGradEngine` - ``(f, grad theta)`` at a given flat parameter vector, the objective
of both L-BFGS variants; also graph-captured on GPU.
"""
from __future__ import annotations

import math
import os
import time

import torch

from .graphs import capture_graph
from .optimizers import adam as adam_mod
from .ops import fused


def _use_graphs(device):
    return (torch.device(device).type == "cuda" and os.environ.get("TDQ_NO_GRAPH", "0") != "1")


class _Bucket:
    """Pack/unpack of the single per-step all-reduce buffer."""

    def __init__(self, tensors, n_scalars):
        self.sizes = [t.numel() for t in tensors]
        self.n_scalars = n_scalars

    def pack(self, grads, scalars):
        return torch.cat([g.reshape(-1) for g in grads] + [s.reshape(1).to(grads[0].dtype) for s in scalars])

    def unpack(self, buf):
        out, off = [], 0
        for n in self.sizes:
            out.append(buf[off:off + n])
            off += n
        return out, buf[off:off + self.n_scalars]   # scal[0] = loss, scal[1:] = terms (contiguous)


def _term_list(terms):
    return list(terms.unbind()) if torch.is_tensor(terms) else list(terms)


class ParamGroup:
    """Tensors updated by one Adam instance.  ``sign=-1``: gradient ascent (SA weights);
    ``reduce[i]``: whether tensor i's gradient is all-reduced under DP (False for sharded SA
    weights, whose gradient is already exact on the owning rank)."""

    def __init__(self, tensors, get_opt, sign=1.0, reduce=None):
        self.tensors = list(tensors)
        self.get_opt = get_opt
        self.sign = float(sign)
        self.reduce = list(reduce) if reduce is not None else [True] * len(self.tensors)


def default_bind(n_lambdas):
    """Map the per-step parameter aliases to ``LossProgram.evaluate`` arguments."""
    def bind(alias):
        return {"params": alias[0], "lambdas": alias[1:1 + n_lambdas]}
    return bind


class AdamEngine:
    """Captured/eager optimizer step.  Gradients are taken w.r.t. fresh
    ``detach().requires_grad_()`` aliases of the parameter buffers (same storage), never the
    persistent leaves: an AccumulateGrad node of a leaf created on the default stream by an
    earlier eager backward would otherwise make autograd sync the legacy null stream inside
    the HIP-graph capture."""

    def __init__(self, solver, program, groups, n_steps_hint=0, lambdas=None, bind=None):
        self.s = solver
        self.program = program
        self.groups = [g for g in groups if g.tensors]
        self.flat = groups[0].tensors[0]
        self.lambdas = lambdas if lambdas is not None else []
        self.dist = solver.dist_ctx
        dev = self.flat.device
        self.device = dev
        self.state = solver._train_state(dev)
        self.term_names = [t.name for t in program.terms]
        self.graph_a = self.graph_b = None
        self.static_loss = None
        self.wrt = [t for g in self.groups for t in g.tensors]
        self.bind = bind if bind is not None else default_bind(len(self.lambdas))
        self.red_idx = [i for i, r in enumerate(r for g in self.groups for r in g.reduce) if r]
        self._bind_opts()
        self._ensure_hist(n_steps_hint)

    def _bind_opts(self):
        """(Re)read optimizer objects - users may replace e.g. ``model.tf_optimizer``."""
        self.opts = [g.get_opt() for g in self.groups]
        self._tail_ok = None
        self.counters = [o.step_counter(self.device) for o in self.opts]
        self.moments = [[o.state_for(t) for t in g.tensors] for o, g in zip(self.opts, self.groups)]

    def _ensure_hist(self, n):
        """Room in the device loss history for ``n`` more steps.  A new buffer invalidates the
        captured step (it writes its row through the buffer's address), so the history grows
        geometrically: repeated short ``fit`` / ``run`` calls re-capture O(log steps) times."""
        st = self.state
        if "improved" not in st:  # allocated here, outside any graph capture
            st["improved"] = torch.zeros((), dtype=torch.int32, device=self.device)
        need = int(st["epoch_host"]) + int(n) + 1
        if st["hist"] is None or st["hist"].shape[0] < need:
            old = 0 if st["hist"] is None else st["hist"].shape[0]
            new = torch.full((max(need, 2 * old, 16), 1 + len(self.term_names)), float("nan"),
                             device=self.device)
            if st["hist"] is not None:
                new[: st["hist"].shape[0]] = st["hist"]
            st["hist"] = new
            self.graph_a = self.graph_b = None  # history pointer changed
            self.graph_k = None

    # ---------------------------------------------------------------- step pieces -------
    def _fused_map(self, fop):
        """wrt index -> where its gradient comes from in the fused kernel outputs."""
        fl = fop.fl
        n_lam = len(self.lambdas)
        src = [("flat", 0)]
        for i in range(1, len(self.wrt)):
            if i <= n_lam:
                k = i - 1
                if k in fl.lam_slots:
                    src.append(("dlam", fl.lam_slots.index(k)))
                elif ("lam", k) in fl.scal_slots:
                    src.append(("dscal", fl.scal_slots.index(("lam", k))))
                else:
                    src.append(("zero", 0))
            else:
                k = i - 1 - n_lam
                src.append(("dscal", fl.scal_slots.index(("extra", k))) if ("extra", k) in fl.scal_slots
                           else ("zero", 0))
        return src

    def _fused_grads(self, fop, gflat, dlam, dscal):
        """Per-wrt-tensor gradients from the fused-loss outputs and the flat theta gradient."""
        if getattr(self, "_fsrc", None) is None:
            self._fsrc = self._fused_map(fop)
        grads = []
        for (kind, k), w in zip(self._fsrc, self.wrt):
            if kind == "flat":
                grads.append(gflat)
            elif kind == "dlam":
                g = dlam[k]
                rng = fop.fl.lam_offsets.get(fop.fl.lam_slots[k])
                if rng is not None:
                    full = torch.zeros(w.numel(), device=w.device)
                    full[rng[0]:rng[1]] = g
                    g = full
                grads.append(g.view_as(w))
            elif kind == "dscal":
                grads.append(dscal[k].view_as(w))
            else:
                grads.append(torch.zeros_like(w))
        return grads

    def _phase_a_fused(self, fop, for_step=False):
        # (Running the loss reduction + bookkeeping on a side stream beside the jet backward was
        # measured slower on MI355X: 0.505 vs 0.494 ms per AC-SA step on one box - the backward
        # holds every SIMD's registers, so the side kernels only delay its workgroups.)
        from .ops import jet_hip
        prog = self.program
        hi = prog.hi_op
        J, saved = jet_hip.forward_raw(prog.X_all, self.flat, prog.net, prog.plan, prog.precision,
                                       rows=fop.fl.n_streams)
        if hi is not None:   # order 3 / 4 streams of the high-order points (ops/jet_hi.py)
            hi.forward(J, self.flat)
        # inside an optimizer step the bookkeeping kernel (fused.step_book) sums the terms
        total, losses, dJ, dlam, dscal = fop(J, with_total=not for_step)
        gflat = jet_hip.backward_raw(saved, dJ)
        if hi is not None:
            gflat = gflat + hi.backward(dJ, self.flat)
        grads = self._fused_grads(fop, gflat, dlam, dscal)
        return total, grads, losses   # losses: contiguous per-term vector

    def _phase_a(self, for_step=False):
        """Loss, gradients (wrt every group tensor) and per-term losses.  ``for_step=True`` (the
        optimizer step paths only): the fused loss leaves the total to the bookkeeping kernel."""
        fop = getattr(self.program, "fused_op", None)
        self._sum_terms = fop is not None and for_step
        if fop is not None:
            return self._phase_a_fused(fop, for_step)
        alias = [t.detach().requires_grad_(True) for t in self.wrt]
        loss, vals = self.program.evaluate(**self.bind(alias))
        grads = torch.autograd.grad(loss, alias, allow_unused=True)
        grads = [torch.zeros_like(w) if g is None else g for g, w in zip(grads, alias)]
        terms = [vals[n].detach().reshape(()) for n in self.term_names]
        return loss.detach(), grads, terms

    def _reduce(self, loss, grads, terms):
        if not self.dist.is_distributed:
            return loss, grads, terms
        red_idx = self.red_idx
        red = [grads[i] for i in red_idx]
        terms = _term_list(terms)
        bucket = _Bucket(red, 1 + len(terms))
        buf = bucket.pack(red, [loss] + terms)
        self.dist.all_reduce_(buf)
        red_out, scal = bucket.unpack(buf)
        grads = list(grads)
        for i, g in zip(red_idx, red_out):
            grads[i] = g.view_as(grads[i])
        return scal[0], grads, scal[1:]

    def _book(self, loss, terms):
        """History row, best tracking, step counters and epoch in one bookkeeping launch."""
        st = self.state
        if "improved" not in st:
            st["improved"] = torch.zeros((), dtype=torch.int32, device=self.device)
        tv = terms if torch.is_tensor(terms) else (
            torch.stack([t.float().reshape(()) for t in terms]) if len(terms)
            else torch.zeros(0, device=self.device))
        fused.step_book(loss, tv.reshape(-1).float().contiguous(), st, self.counters,
                        sum_terms=getattr(self, "_sum_terms", False))

    def _opt_groups(self, grads):
        """``fused.adam_multi_opts`` rows: each group with its optimizer's counter and
        hyper-parameters."""
        off = 0
        opt_groups = []
        for grp, opt, t, mom in zip(self.groups, self.opts, self.counters, self.moments):
            n = len(grp.tensors)
            items = [(p, g, m, v, grp.sign) for p, g, (m, v) in zip(grp.tensors, grads[off:off + n], mom)]
            opt_groups.append((items, t, opt.learning_rate, opt.beta_1, opt.beta_2, opt.epsilon))
            off += n
        return opt_groups

    def _phase_b(self, loss, grads, terms):
        """Bookkeeping (``fused.step_book``: history row, best tracking, step counters, epoch),
        then ONE Adam launch for every group (each with its optimizer's counter and
        hyper-parameters), which also snapshots the best weights (before the update) when the
        step improved the loss."""
        st = self.state
        self._book(loss, terms)
        opt_groups = self._opt_groups(grads)
        # theta descent + SA-weight ascent in one launch; it also snapshots the best weights
        snap = (st["best_flat"], st["improved"]) if self.groups[0].tensors[0] is self.flat else None
        fused.adam_multi_opts(opt_groups, snapshot=snap)
        return loss

    # ------------------------------------------------------------ fused step tail ------
    def _tail_eligible(self):
        """Step on the split-bf16 jet kernels with the fused loss: single-process, the end of the
        step runs as two launches (csrc/jet_bf3.hip ``tdq_step_tail_bf3``); under DP the captured
        halves use ``tdq_dp_tail_a_bf3`` / ``tdq_dp_tail_b_bf3`` around the all-reduce."""
        if getattr(self, "_tail_ok", None) is not None:
            return self._tail_ok
        ok = False
        fop = getattr(self.program, "fused_op", None)
        if (os.environ.get("TDQ_FUSED_TAIL", "1") != "0" and fop is not None
                and self.device.type == "cuda" and self.groups[0].tensors[0] is self.flat):
            from .ops import _lib, jet_hip
            from .ops.jet_mlp import hip_config
            prog = self.program
            try:
                ok = jet_hip.is_split_bf16(hip_config(prog.net, prog.plan, prog.precision)) and _lib.available()
            except (ValueError, AttributeError):
                ok = False
            if ok:
                probe = [(w, w, m, v, 1.0) for w, (m, v) in zip(self.wrt, (mv for ms in self.moments for mv in ms))]
                ok = fused.group_array([(probe, self.counters[0], 0.0, 0.0, 0.0, 0.0)]) is not None
        self._tail_ok = ok
        return ok

    def _step_buffers(self):
        """Jets, forward scratch (saved activations + weight images), gradient slabs and the
        theta gradient of the fused-tail step, allocated once per engine."""
        if getattr(self, "_bufs", None) is None:
            from .ops import jet_hip
            prog = self.program
            J, saved = jet_hip.alloc_forward(prog.X_all, self.flat, prog.net, prog.plan, prog.precision,
                                             rows=prog.fused_op.fl.n_streams)
            self._bufs = (J, saved, jet_hip.alloc_backward(saved), torch.empty_like(self.flat))
        return self._bufs

    def _fused_step(self):
        """The one-launch residual step (ops/fused_step.py) or None."""
        from .ops import fused_step
        return fused_step.for_program(self.program)

    def _point_ranges(self, fop):
        if getattr(self, "_ranges", 0) == 0:
            self._ranges = point_ranges(self.program, fop)
            self._streams = [torch.cuda.Stream(device=self.device) for _ in (self._ranges or ())]
        return self._ranges

    def _tail_step(self, in_graph):
        """One Adam step ending in the fused tail.  ``in_graph``: the step is being captured, so
        the forward reuses the weight images that the previous replay's tail wrote (the engine
        re-packs them once before the first replay of every :meth:`run`)."""
        from .ops import jet_hip
        prog = self.program
        fop = prog.fused_op
        st = self.state
        if "improved" not in st:
            st["improved"] = torch.zeros((), dtype=torch.int32, device=self.device)
        if st["best_flat"].numel() != self.flat.numel():
            raise ValueError(f"best-weights snapshot has {st['best_flat'].numel()} elements, parameters "
                             f"{self.flat.numel()}")
        # persistent buffers: every captured step (the 1-step and the K-step graph) reads the weight
        # images the previous step's tail wrote into this one scratch
        J, saved, work, grad = self._step_buffers()
        pre, kw = self._run_points(J, saved, work, pack=not in_graph)
        grads = self._fused_grads(fop, grad, fop.dlam, fop.dscal)
        packed = fused.group_array(self._opt_groups(grads))
        if packed is None:  # gradient tensors the single launch cannot take: reduce, then Adam
            raise RuntimeError("fused step tail: parameter groups do not fit one launch "
                               "(set TDQ_FUSED_TAIL=0)")
        hi = prog.hi_op
        jet_hip.step_tail(saved, work, grad, fop, st, self.counters, packed[0], packed[1], st["best_flat"],
                          write_images=in_graph, c_first=pre, gextra=hi.grad if hi is not None else None, **kw)
        self._tail_saved = saved
        return fop.total

    def _run_points(self, J, saved, work, pack):
        """Gradient slabs + loss partials of every point: the fused residual step beside the
        boundary chain, else the point ranges' forward -> loss -> backward chains.  Returns
        ``(first slab chunk of the tail, tail keyword arguments)``."""
        prog, fop = self.program, self.program.fused_op
        fs = self._fused_step()
        if fs is not None:
            fs.run(saved, J, work, self.flat, pack=pack)
            return 0, fs.tail_kw()
        rng = self._point_ranges(fop) or [(0, prog.X_all.shape[0], 0, fop.n_blocks)]
        pre = prereduce_chunk(prog, rng)
        run_ranges(prog, fop, self.flat, rng, self._streams, pack=pack, bufs=(J, saved, work), prereduce=pre)
        return pre, {}

    def _dp_tail_phase_b(self, loss, grads, terms):
        """DP graph half after the all-reduce: bookkeeping, then Adam + snapshot + weight images."""
        from .ops import jet_hip
        st = self.state
        self._book(loss, terms)
        if st["best_flat"].numel() != self.flat.numel():
            raise ValueError(f"best-weights snapshot has {st['best_flat'].numel()} elements, parameters "
                             f"{self.flat.numel()}")
        packed = fused.group_array(self._opt_groups(grads))
        if packed is None:
            raise RuntimeError("fused step tail: parameter groups do not fit one launch "
                               "(set TDQ_FUSED_TAIL=0)")
        jet_hip.dp_tail_b(self._tail_saved, packed[0], packed[1], st["improved"], st["best_flat"])
        return loss

    def _eager_step(self):
        if self._tail_eligible():
            if not self.dist.is_distributed:
                return self._tail_step(in_graph=False)
            # DP: the captured step's own sequence, eagerly (same kernels, so the warm-up step and
            # the replays share one numerics - the fused step's bf16 kernels)
            self._dp_half_a_inplace(pack=True)
            self.dist.all_reduce_(self._bucket_buf)
            self._dp_half_b(True)
            return self.static_loss
        loss, grads, terms = self._phase_a(for_step=True)
        loss, grads, terms = self._reduce(loss, grads, terms)
        return self._phase_b(loss, grads, terms)

    # ---------------------------------------------------------------- graphs -------------
    def _capture(self):
        if self._tail_eligible():
            self._fused_step()   # built (hipRTC compile + module load) outside any capture
        stream = torch.cuda.Stream(device=self.device)
        stream.wait_stream(torch.cuda.current_stream(self.device))
        split = self.dist.is_distributed
        with torch.cuda.stream(stream):
            # warm-up: one real (counted) step on the side stream
            warm = self._eager_step()
            self.state["epoch_host"] += 1
        torch.cuda.current_stream(self.device).wait_stream(stream)
        torch.cuda.synchronize(self.device)
        pool = torch.cuda.graph_pool_handle()
        self._graph_saved = None
        if not split:
            tail = self._tail_eligible()
            g = torch.cuda.CUDAGraph()
            with capture_graph(g, pool=pool):
                self.static_loss = self._tail_step(in_graph=True) if tail else self._eager_step()
            self.graph_a, self.graph_b = g, None
            if tail:
                self._graph_saved = self._tail_saved
        else:
            tail = self._tail_eligible()
            self.dist.settle_collective(self._bucket_floats())
            if self._coll_in_graph():
                # RCCL: the bucket all-reduce is captured in the step graph - one replay per step
                g = torch.cuda.CUDAGraph()
                with capture_graph(g, pool=pool):
                    self._dp_half_a(tail)
                    self.dist.all_reduce_(self._bucket_buf)
                    self._dp_half_b(tail)
                self.graph_a, self.graph_b = g, None
            else:
                ga = torch.cuda.CUDAGraph()
                with capture_graph(ga, pool=pool):
                    self._dp_half_a(tail)
                gb = torch.cuda.CUDAGraph()
                with capture_graph(gb, pool=pool):
                    self._dp_half_b(tail)
                self.graph_a, self.graph_b = ga, gb
            if tail:
                self._graph_saved = self._tail_saved
        return warm

    def _dp_half_a(self, tail):
        """DP step up to the collective: loss + gradients, packed into the static bucket."""
        if tail:
            return self._dp_half_a_inplace()
        loss, grads, terms = self._phase_a(for_step=True)
        red_idx = self.red_idx
        red = [grads[i] for i in red_idx]
        terms = _term_list(terms)
        self._bucket = _Bucket(red, 1 + len(terms))
        self._bucket_buf = self._bucket.pack(red, [loss] + terms)
        self._grads_static = grads
        self._red_idx = red_idx

    def _dp_half_a_inplace(self, pack=False):
        """Fused-tail DP step up to the collective with the kernels writing straight into the
        bucket ``[grad theta | other reduced grads | loss | terms]``: slab pass 2 lands in the
        theta slice, the loss reduction in the scalar slice, so only the (small) other reduced
        gradients are copied - no concatenation of the 50k-element theta gradient per step."""
        from .ops import jet_hip
        prog = self.program
        fop = prog.fused_op
        # persistent step buffers (as in _tail_step): the 1-step and the K-step graph read the
        # weight images that the previous step's dp_tail_b wrote into this one scratch
        J, saved, work, _ = self._step_buffers()
        pre, kw = self._run_points(J, saved, work, pack=pack)
        n_p = self.flat.numel()
        red_idx = self.red_idx
        if not red_idx or red_idx[0] != 0:
            raise RuntimeError("DP bucket: theta must be the first reduced tensor")
        others = [i for i in red_idx[1:]]
        sizes = [self.wrt[i].numel() for i in others]
        n_e, n_t = sum(sizes), fop.n_terms
        buf = getattr(self, "_dp_buf", None)
        if buf is None or buf.numel() != n_p + n_e + 1 + n_t:
            buf = self._dp_buf = torch.empty(n_p + n_e + 1 + n_t, dtype=torch.float32, device=self.device)
        grad_view = buf[:n_p]
        hi = prog.hi_op
        jet_hip.dp_tail_a(saved, work, grad_view, fop, total=buf[n_p + n_e:n_p + n_e + 1],
                          losses=buf[n_p + n_e + 1:], c_first=pre, gextra=hi.grad if hi is not None else None, **kw)
        grads = self._fused_grads(fop, grad_view, fop.dlam, fop.dscal)
        if others:
            torch.cat([grads[i].reshape(-1) for i in others], out=buf[n_p:n_p + n_e])
        self._sum_terms = True
        self._tail_saved = saved
        self._bucket = _Bucket([grads[i] for i in red_idx], 1 + n_t)
        self._bucket_buf = buf
        self._grads_static = grads
        self._red_idx = red_idx

    def _dp_half_b(self, tail):
        """DP step after the collective: unpack the bucket, bookkeeping, optimizer update."""
        red_out, scal = self._bucket.unpack(self._bucket_buf)
        grads = list(self._grads_static)
        for i, gg in zip(self._red_idx, red_out):
            grads[i] = gg.view_as(grads[i])
        self.static_loss = (self._dp_tail_phase_b if tail else self._phase_b)(scal[0], grads, scal[1:])

    def _capture_k(self, k):
        """K fused-tail steps in ONE graph (single process): replays of a 1-step graph leave the
        GPU idle ~9 us between graphs (rocprofv3 kernel trace, tools/timeline.py); inside a
        graph the steps follow back to back.  Every step's state lives on the device (epoch,
        history row, counters, best tracking), so K captured copies are K real steps."""
        pool = torch.cuda.graph_pool_handle()
        g = torch.cuda.CUDAGraph()
        with capture_graph(g, pool=pool):
            for _ in range(k):
                if self.dist.is_distributed:   # graph_collectives: the all-reduce is a graph node
                    self._dp_half_a(True)
                    self.dist.all_reduce_(self._bucket_buf)
                    self._dp_half_b(True)
                    loss = self.static_loss
                else:
                    loss = self._tail_step(in_graph=True)
        self.graph_k, self.static_loss_k, self._k = g, loss, k

    def _bucket_floats(self):
        """Upper bound of the per-step DP bucket: every reduced gradient + loss + terms."""
        return sum(self.wrt[i].numel() for i in self.red_idx) + 1 + len(self.term_names)

    def _coll_in_graph(self):
        """Capture the bucket all-reduce inside the step graph (RCCL, or the peer kernel when it
        takes a bucket of this size; ADVICE r3: a gloo fallback must never be captured)."""
        return self.dist.capturable(self._bucket_floats())

    def _replay(self):
        self.graph_a.replay()
        if self.graph_b is not None:
            self.dist.all_reduce_(self._bucket_buf)
            self.graph_b.replay()
        return self.static_loss

    # ---------------------------------------------------------------- driver -------------
    def run(self, n_steps, progress=None, log_every=100, use_graph=None):
        """Run ``n_steps`` optimizer steps; returns the last loss (device tensor)."""
        if n_steps <= 0:
            return None
        opts = [g.get_opt() for g in self.groups]
        sig = [(o.learning_rate, o.beta_1, o.beta_2, o.epsilon) for o in opts]
        if any(a is not b for a, b in zip(opts, self.opts)) or sig != getattr(self, "_sig", sig):
            self._bind_opts()
            self.graph_a = self.graph_b = None
            self.graph_k = None
        self._sig = sig
        self._ensure_hist(n_steps)
        use_graph = _use_graphs(self.device) if use_graph is None else use_graph
        st = self.state
        loss = None
        done = 0
        if use_graph and self.graph_a is None:
            loss = self._capture()
            done = 1
            if progress is not None and n_steps == 1:
                progress(1, float(loss))
        if use_graph and self.graph_a is not None and getattr(self, "_graph_saved", None) is not None \
                and done < n_steps:
            # the captured step's forward reads weight images written by the previous replay's
            # tail: bring them up to date with the parameters as they are now
            from .ops import jet_hip
            jet_hip.pack_images(self._graph_saved)
        checked = int(st["epoch_host"]) - done
        K = self._unroll()
        if use_graph and self.graph_a is not None and K > 1 and n_steps - done >= K \
                and getattr(self, "graph_k", None) is None:
            self._capture_k(K)
        while done < n_steps:
            # K steps at once unless that would jump over a progress / NaN-check point
            next_log = (done // log_every + 1) * log_every if progress is not None else n_steps
            if use_graph and K > 1 and getattr(self, "graph_k", None) is not None and n_steps - done >= K \
                    and done + K <= next_log:
                self.graph_k.replay()
                loss = self.static_loss_k
                done += K
                st["epoch_host"] += K
            else:
                loss = self._replay() if (use_graph and self.graph_a is not None) else self._eager_step()
                done += 1
                st["epoch_host"] += 1
            if progress is not None and (done % log_every == 0 or done == n_steps):
                checked = self._check_finite(checked)
                progress(done, float(loss))
        self._check_finite(checked)
        return loss

    def _unroll(self):
        """Steps per multi-step graph (``TDQ_STEP_UNROLL``, default 8): fused-tail steps, single
        process or DP with the all-reduce captured in the graph (RCCL / peer); 1 = one graph per
        step."""
        if not self._tail_eligible() or (self.dist.is_distributed and not self._coll_in_graph()):
            return 1
        return max(1, int(os.environ.get("TDQ_STEP_UNROLL", "8")))

    def _check_finite(self, lo):
        """Failure detection: the loss-history rows ``[lo, epoch)`` written on the
        device by the captured steps are scanned with one reduction and one read-back, at the
        progress cadence and at the end of every :meth:`run` - never inside the step.  A NaN / Inf
        total loss raises ``FloatingPointError`` naming the first bad epoch (the best-weights
        snapshot, taken before each update, still holds the last finite model).  ``TDQ_NAN_CHECK=0``
        disables the check.  Returns the new low-water mark."""
        st = self.state
        hi = int(st["epoch_host"])
        self.dist.check_health()
        if hi <= lo or os.environ.get("TDQ_NAN_CHECK", "1") == "0":
            return hi
        col = st["hist"][lo:hi, 0]
        # fast path: one reduction + one read-back (a NaN / Inf anywhere makes the sum non-finite;
        # a finite-but-overflowing sum falls through to the exact scan, which then finds nothing)
        if math.isfinite(float(col.sum())):
            return hi
        bad = ~torch.isfinite(col)
        if bool(bad.any()):
            first = lo + int(torch.nonzero(bad)[0, 0])
            raise FloatingPointError(f"Adam: loss became {float(st['hist'][first, 0])} at epoch {first} "
                                     f"(best finite loss {float(st['best_loss']):.6g} at epoch "
                                     f"{int(st['best_epoch'])}; predict(best_model=True) uses it)")
        return hi


def point_ranges(program, fop):
    """Point ranges whose forward -> loss -> backward chains run on separate streams (graph
    branches), or ``None``.

    One jet launch over N points is a whole number of wave rounds (bf16 at 50k points: 3184 waves
    of 16 points over 2048 wave slots = 1.55 rounds, run as 2; bf16x3: 3.1 rounds over 1024 slots,
    run as 4), and the loss launch between them idles the GPU.  With the points in two ranges on
    two streams, the loss and backward of one range fill the slots the forward of the other
    leaves idle (MI355X, AC-SA 50k: bf16 Adam step 0.211 -> 0.200 ms, bf16x3 0.446 -> 0.411 ms,
    bf16x3 L-BFGS iteration 0.51 -> 0.48 ms; profiles/r3_l_split_sweep.jsonl).  ``TDQ_SPLIT``:
    ``auto`` (default: cut at 0.38 for bf16, 0.35 for bf16x3, the sweeps' best), ``0`` / ``off``,
    or the cut fraction.  Cuts land on multiples of 128 points that also cut the fused loss's blocks
    cleanly (:meth:`FusedLossOp.split_block`); results are bitwise those of single launches (every
    workgroup / block keeps its index and buffers)."""
    from .ops.jet_mlp import hip_config
    spec = os.environ.get("TDQ_SPLIT", "auto").strip().lower()
    if spec in ("0", "off", "none", "", "0.0"):
        return None
    try:
        cfg = hip_config(program.net, program.plan, program.precision)
    except ValueError:
        return None
    if cfg["precision"] not in ("bf16x3", "bf16") or cfg.get("engine") == "layered":
        return None
    from .ops import jet_hip
    if spec == "auto":
        # sweeps on MI355X with the specialized loss kernel: bf16 0.38 (0.2018 ms vs 0.2035 at 0.45,
        # 3 passes, profiles/r3_yz_split_sweep_jit.jsonl), bf16x3 0.30-0.40 equal within noise.
        # Mixed programs (high-order kernels on the first range's stream): the first range the
        # LONGER one, 0.62 (AC-baseline 0.231-0.232 ms vs 0.251-0.261 at 0.30-0.55,
        # profiles/r4s_place.jsonl) - its high-order gradient then overlaps the other range's backward
        if getattr(program, "hi_op", None) is not None:
            fracs = [0.62]
        else:
            fracs = [0.35] if cfg["precision"] == "bf16x3" else [0.38]
    else:
        fracs = sorted(float(v) for v in spec.split(","))
    if len(fracs) > 1:
        # three graph branches made hipGraphLaunch segfault on the host (ROCm 7.2, MI355X,
        # gpurun_out r3l); two are tested (tests/test_hip_kernels.py, tests/test_dist_gpu.py)
        raise ValueError("TDQ_SPLIT: one cut (two point ranges) at most")
    N = program.X_all.shape[0]
    if N < 8192:
        return None
    # preferred cuts: a row boundary of the slab reduction's chunks (slab_chunk_lo), so the first
    # range's rows are pre-reduced while the second range's backward runs (prereduce_chunk) with
    # every summation order unchanged; else the nearest multiple of 128 points
    try:
        pts_b, nwg, chunks, _ = jet_hip.slab_geometry(cfg, N)
        bounds = [(nwg * c // chunks) * pts_b for c in range(1, chunks)]
        bounds = [a for a in bounds if a % 128 == 0]
    except Exception:  # noqa: BLE001 - no native library: plain 128-point cuts
        bounds = []
    cuts, blks = [0], [0]
    for f in fracs:
        b = None
        cands = ([min(bounds, key=lambda a: abs(a - f * N))] if bounds else []) + [int(round(f * N / 128)) * 128]
        for a in cands:
            if cuts[-1] < a < N and abs(a - f * N) <= 0.05 * N:
                b = fop.split_block(a)
                if b is not None and b > blks[-1]:
                    break
            b = None
        if b is None:
            return None
        cuts.append(a)
        blks.append(b)
    cuts.append(N)
    blks.append(fop.n_blocks)
    return [(cuts[i], cuts[i + 1], blks[i], blks[i + 1] - blks[i]) for i in range(len(cuts) - 1)]


def prereduce_chunk(program, ranges):
    """First-pass chunk index at the cut between two point ranges when the cut lies on a chunk
    boundary of the slab reduction (those chunks are reduced right after the first range's
    backward), else 0."""
    if not ranges or len(ranges) != 2 or os.environ.get("TDQ_PREREDUCE", "1") == "0":
        return 0
    from .ops import jet_hip
    from .ops.jet_mlp import hip_config
    cfg = hip_config(program.net, program.plan, program.precision)
    pts_b, nwg, chunks, _ = jet_hip.slab_geometry(cfg, program.X_all.shape[0])
    cut = ranges[0][1]
    for c in range(1, chunks):
        if (nwg * c // chunks) * pts_b == cut:
            return c
    return 0


def run_ranges(program, fop, flat, ranges, streams, pack=True, bufs=None, prereduce=0):
    """Forward -> fused loss -> backward of every point range, each range on its own stream
    (forked from and joined back into the current one; one range runs on the current stream).
    ``bufs``: ``(J, saved, work)`` to reuse (persistent step buffers), else allocated here.
    ``prereduce`` (> 0): after the first range's backward, reduce slab chunks ``[0, prereduce)`` on
    its stream (the fused step tail then starts at that chunk).  Mixed programs (``program.hi_op``):
    the high-order points ``[0, n_hi)`` lie in the first range, whose chain also runs their extra
    streams (before its loss launch) and the gradient of those streams' adjoints (after it) - off
    the longer second range's critical path.  Returns ``(saved, work)`` for the fused step tail."""
    from .ops import jet_hip
    hop = program.hi_op
    if bufs is None:
        J, saved = jet_hip.alloc_forward(program.X_all, flat, program.net, program.plan, program.precision,
                                         rows=fop.fl.n_streams)
        work = jet_hip.alloc_backward(saved)
    else:
        J, saved, work = bufs
    if pack:
        jet_hip.pack_images(saved)
    if hop is not None and ranges[0][1] < program.n_hi:
        raise RuntimeError("point ranges: the first range must hold the high-order points")
    cur = torch.cuda.current_stream(flat.device)
    # the high-order points' extra streams (a hundred workgroups of long per-layer chains; they
    # touch only their own J rows) run on range 0's stream: their forward before range 0's forward,
    # their gradient between its loss and its backward - with range 0 the longer range
    # (point_ranges) that gradient runs beside range 1's backward.  AC-baseline step on MI355X:
    # 0.231-0.237 ms at cut 0.62; the other placements measured in round 4 (gradient after the
    # backward, forward on a third graph branch, the two pieces across the branches, the gradient
    # split between them) were equal or slower - profiles/r4l_place.jsonl, r4q_place_cut_sweep.jsonl,
    # r4s_place.jsonl, r4u_*, r4split_* - and were removed.

    def chain(k, lo, hi, b0, nb):
        if k == 0 and hop is not None:
            hop.forward(J, flat)
        jet_hip.forward_range(saved, J, lo, hi)
        fop.run_range(J, b0, nb)
        if k == 0 and hop is not None:
            hop.backward(fop.dJ, flat)
        jet_hip.backward_range(saved, fop.dJ, work, lo, hi)
        if k == 0 and prereduce:
            jet_hip.slab_prereduce(saved, work, 0, prereduce)

    if len(ranges) == 1:
        chain(0, *ranges[0])
        return saved, work
    # (keeping one range on the current stream measured the same: the graph runtime picks the
    # hardware queues of its branches itself, and the join still waits ~9 us across queues)
    for st in streams[:len(ranges)]:
        st.wait_stream(cur)
    for k, ((lo, hi, b0, nb), st) in enumerate(zip(ranges, streams)):
        with torch.cuda.stream(st):
            chain(k, lo, hi, b0, nb)
    for st in streams[:len(ranges)]:
        cur.wait_stream(st)
    return saved, work


class LossGradEngine:
    """``(f, g_theta)`` at a flat parameter vector (lambdas frozen, B15); DP all-reduced."""

    def __init__(self, solver, program, lambdas):
        self.s = solver
        self.program = program
        self.flat = solver.u_model.flat
        self.lambdas = lambdas
        self.dist = solver.dist_ctx
        self.graph = None
        self.n_evals = 0

    def _fused_tail(self):
        """Split-bf16 kernels with the fused loss on a GPU: ``[grad | loss]`` is written in place
        by the fused tail (slab pass 1 + loss reduction + total in one launch, slab pass 2 into the
        buffer) instead of loss-reduce / total / slab / concatenate launches."""
        ok = getattr(self, "_tail", None)
        if ok is None:
            ok = False
            if os.environ.get("TDQ_FUSED_TAIL", "1") != "0" and self.flat.is_cuda:
                from .ops import _lib, jet_hip
                from .ops.jet_mlp import hip_config
                prog = self.program
                try:
                    ok = jet_hip.is_split_bf16(hip_config(prog.net, prog.plan, prog.precision)) and _lib.available()
                except (ValueError, AttributeError):
                    ok = False
            self._tail = ok
        return ok

    def _fused_bufs(self):
        """Persistent forward / backward buffers of the one-launch objective."""
        if getattr(self, "_fbufs", None) is None:
            from .ops import jet_hip
            prog = self.program
            J, saved = jet_hip.alloc_forward(prog.X_all, self.flat, prog.net, prog.plan, prog.precision,
                                             rows=prog.fused_op.fl.n_streams)
            self._fbufs = (J, saved, jet_hip.alloc_backward(saved))
        return self._fbufs

    def image_target(self):
        """``(img_target, evaluate_fg without the pack launch)`` when the objective is the
        one-launch fused step (its weight images can be written by the optimizer's own update
        kernel, csrc/lbfgs.hip), else ``None``."""
        fop = getattr(self.program, "fused_op", None)
        if fop is None or not self._fused_tail() or getattr(self.program, "hi_op", None) is not None:
            return None
        from .ops import fused_step, jet_hip
        if fused_step.for_program(self.program) is None:
            return None
        return jet_hip.img_target(self._fused_bufs()[1]), (lambda: self._body(pack=False))

    def _body(self, pack=True):
        fop = getattr(self.program, "fused_op", None)
        if fop is not None:
            from .ops import jet_hip
            prog = self.program
            if self._fused_tail():
                fg = torch.empty(self.flat.numel() + 1, dtype=torch.float32, device=self.flat.device)
                if getattr(self, "_ranges", 0) == 0:
                    self._ranges = point_ranges(prog, fop)
                    self._streams = [torch.cuda.Stream(device=self.flat.device) for _ in (self._ranges or ())]
                hi = prog.hi_op
                gx = hi.grad if hi is not None else None
                from .ops import fused_step
                # the one-launch objective (bf16: jet_fused.h, bf16x3: jet_fused3.h) on persistent
                # buffers (the image target of the device L-BFGS points into their scratch)
                fs = fused_step.for_program(prog)
                if fs is not None:
                    J, saved, work = self._fused_bufs()
                    fs.run(saved, J, work, self.flat, pack=pack)
                    jet_hip.dp_tail_a(saved, work, fg[:-1], fop, total=fg[-1:], gextra=gx, **fs.tail_kw())
                    return fg
                if self._ranges:
                    pre = prereduce_chunk(prog, self._ranges)
                    saved, work = run_ranges(prog, fop, self.flat, self._ranges, self._streams, prereduce=pre)
                    jet_hip.dp_tail_a(saved, work, fg[:-1], fop, total=fg[-1:], c_first=pre, gextra=gx)
                    return fg
                J, saved = jet_hip.forward_raw(prog.X_all, self.flat, prog.net, prog.plan, prog.precision,
                                               rows=fop.fl.n_streams)
                if hi is not None:
                    hi.forward(J, self.flat)
                fop(J, with_total=False, reduce=False)
                if hi is not None:
                    hi.backward(fop.dJ, self.flat)
                grad, work = jet_hip.backward_raw(saved, fop.dJ, reduce=False, grad=fg[:-1])
                jet_hip.dp_tail_a(saved, work, grad, fop, total=fg[-1:], gextra=gx)
                return fg
            hi = prog.hi_op
            J, saved = jet_hip.forward_raw(prog.X_all, self.flat, prog.net, prog.plan, prog.precision,
                                           rows=fop.fl.n_streams)
            if hi is not None:
                hi.forward(J, self.flat)
            total, _, dJ, _, _ = fop(J)
            g = jet_hip.backward_raw(saved, dJ)
            if hi is not None:
                g = g + hi.backward(dJ, self.flat)
            return torch.cat([g.reshape(-1), total.reshape(1)])
        p = self.flat.detach().requires_grad_(True)
        lams = [l.detach() for l in self.lambdas]
        loss, _ = self.program.evaluate(p, lams)
        g = torch.autograd.grad(loss, [p])[0]
        buf = torch.cat([g.reshape(-1), loss.detach().reshape(1)])
        return buf

    def evaluate_fg(self):
        """``[grad | loss]`` at the CURRENT flat parameters (nothing copied in, not all-reduced):
        the objective of the device L-BFGS, captured inside its HIP graph."""
        return self._body()

    def __call__(self, x):
        with torch.no_grad():
            self.flat.copy_(x)
        use_graph = _use_graphs(self.flat.device)
        # the all-reduce is captured with the evaluation (RCCL, or the peer kernel if it takes
        # the [grad | loss] buffer)
        in_graph = self.dist.capturable(self.flat.numel() + 1)
        if use_graph and self.graph is None and self.n_evals >= 1:
            stream = torch.cuda.Stream(device=self.flat.device)
            stream.wait_stream(torch.cuda.current_stream(self.flat.device))
            with torch.cuda.stream(stream):
                self._body()
            torch.cuda.current_stream(self.flat.device).wait_stream(stream)
            g = torch.cuda.CUDAGraph()
            with capture_graph(g):
                self._static = self._body()
                if in_graph:
                    self.dist.all_reduce_(self._static)
            self.graph = g
        if self.graph is not None:
            self.graph.replay()
            buf = self._static.clone()
            reduced = in_graph
        else:
            buf = self._body()
            reduced = False
        self.n_evals += 1
        if self.dist.is_distributed and not reduced:
            self.dist.all_reduce_(buf)
        if in_graph and self.dist.peer is not None and self.n_evals % 32 == 0:
            # a peer all-reduce that timed out inside the replayed graph summed stale slots: raise
            # instead of handing the optimizer a corrupted gradient
            self.dist.check_health()
        return buf[-1], buf[:-1]


class Timer:
    def __init__(self, device):
        self.device = torch.device(device)

    def sync(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def __enter__(self):
        self.sync()
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        self.sync()
        self.elapsed = time.perf_counter() - self.t0
        return False


def nan_guard(loss, where="loss"):
    """Host-side check of one scalar (the L-BFGS wrappers; the Adam engine scans its device
    history instead, :meth:`AdamEngine._check_finite`)."""
    v = float(loss)
    if math.isnan(v) or math.isinf(v):
        raise FloatingPointError(f"{where} became {v}")
    return v


# ---- reference functional API (tensordiffeq/fit.py) ------------------------------------------
def fit(obj, tf_iter=0, newton_iter=0, batch_sz=None, newton_eager=True):
    """Functional form of :meth:`CollocationSolverND.fit` (reference ``fit.py:17-102``): Adam for
    ``tf_iter`` steps (graph-captured fused step), then L-BFGS for ``newton_iter`` iterations."""
    return obj.fit(tf_iter=tf_iter, newton_iter=newton_iter, batch_sz=batch_sz, newton_eager=newton_eager)


def fit_dist(obj, tf_iter=0, newton_iter=0, batch_sz=None, newton_eager=True):
    """Data-parallel fit (reference ``fit.py:150-224``).  ``obj`` must be compiled with ``dist=True``
    under torchrun (one process per GPU); points and SA weights are sharded, one flat all-reduce per
    step.  Unlike the reference, L-BFGS also runs under DP and repeated calls resume (B6, B7)."""
    if not getattr(obj, "dist", False):
        raise ValueError("fit_dist needs a solver compiled with dist=True (launch with torchrun)")
    return obj.fit(tf_iter=tf_iter, newton_iter=newton_iter, batch_sz=batch_sz, newton_eager=newton_eager)


def train_op_inner(obj):
    """One optimizer step: Adam descent on the network, Adam ascent on the SA weights
    (reference ``fit.py:125-147``).  Returns the loss before the step (device scalar)."""
    eng = obj._get_engine(None, 1)
    return eng.run(1, use_graph=False)


def lbfgs_train(obj, newton_iter=100):
    """Strong-Wolfe L-BFGS on the network parameters (the reference's TFP graph path,
    ``fit.py:107-112``); SA weights stay frozen (B15).  The final iterate is kept (B10)."""
    obj._fit_lbfgs(newton_iter, newton_eager=False)
    return obj.min_loss["l-bfgs"]


def lbfgs_op(func, init_params, newton_iter):
    """Minimise ``func(x) -> (loss, grad)`` from ``init_params`` (reference ``fit.py:115-122``,
    ``tfp.optimizer.lbfgs_minimize`` with tolerance 1e-20).  Returns ``(x, loss)``."""
    from .optimizers.lbfgs import graph_lbfgs
    return graph_lbfgs(func, init_params, newton_iter)
