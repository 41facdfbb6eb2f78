"""``DiscoveryModel`` - inverse problems: learn PDE coefficients from observations.

Reference: tensordiffeq/models.py:324-396.  ``compile(layer_sizes, f_model, X, u, var,
col_weights=None)`` with ``f_model(u_model, var, *X)``; loss ``MSE(u(X), u*) + MSE(f, 0)`` or,
with self-adaptive collocation weights, ``MSE(u(X), u*) + mean(col_weights^2 f^2)``; three Adam
instances (network, coefficients, weights - the weights by gradient ascent).

Fixed: the reference never updated the last output bias (``grads[:-(len_+2)]`` truncation,
B22) - every parameter trains here.  The observation points are served by the same single jet
evaluation as the residual (one HIP jet pass covers u and every derivative the residual needs),
and data parallelism shards the observations.

Added: ``fit(tf_iter, newton_iter)`` - after Adam, L-BFGS over the network AND the coefficients
(collocation weights frozen, as the forward solver freezes its SA weights, B15).  Adam moves a
scalar coefficient by ~lr per step whatever its gradient, so at the reference's lr 5e-3 it cannot
resolve c1 = 1e-4 of the Allen-Cahn example (the reference notes "doesnt work quite yet",
examples/AC-discovery.py:68); the quasi-Newton phase has no such floor.
"""
from __future__ import annotations

import numpy as np
import torch
from tqdm.auto import tqdm

from ..fit import AdamEngine, ParamGroup
from ..optimizers import Adam
from ..output import print_screen
from ..parallel import dist as pdist
from .collocation import default_device
from .loss import LossProgram, Term
from .networks import TanhMLP


def Variable(value, dtype=torch.float32, device=None):
    """Trainable scalar/tensor (stand-in for ``tf.Variable`` in discovery examples)."""
    t = torch.as_tensor(value, dtype=dtype)
    if device is not None:
        t = t.to(device)
    return t.detach().clone().requires_grad_(True)


class DiscoveryModel:
    def __init__(self, verbose=True):
        self.verbose = verbose
        self._engine = None
        self._program = None
        self._state = None
        self.log_every = 100
        self.var_history = []

    def compile(self, layer_sizes, f_model, X, u, var, col_weights=None, dist=False,
                backend="auto", device=None, seed=None, precision=None, newton_precision=None, lbfgs_stop=None):
        if seed is not None:
            from ..utils.seeding import set_seed
            set_seed(seed)
        self.dist_ctx = pdist.init_distributed(auto_launch=True) if dist else pdist.get_context(device)
        self.device = torch.device(device) if device is not None else (
            self.dist_ctx.device if dist else default_device())
        ctx = self.dist_ctx
        self.layer_sizes = list(layer_sizes)
        self.f_model = f_model
        cols = [np.reshape(np.asarray(x.detach().cpu() if torch.is_tensor(x) else x), (-1, 1)) for x in X]
        Xm = np.hstack(cols).astype(np.float32)
        self.N = Xm.shape[0]
        self._lo, self._hi = pdist.shard_range(self.N, ctx.rank, ctx.world)
        self.X = torch.as_tensor(Xm[self._lo:self._hi], device=self.device)
        self.X_in = tuple(self.X[:, j:j + 1] for j in range(self.X.shape[1]))
        uu = np.reshape(np.asarray(u.detach().cpu() if torch.is_tensor(u) else u), (-1, 1)).astype(np.float32)
        self.u = torch.as_tensor(uu[self._lo:self._hi], device=self.device)
        self.vars = [v if (torch.is_tensor(v) and v.requires_grad and v.device == self.device)
                     else Variable(v.detach().cpu() if torch.is_tensor(v) else v, device=self.device)
                     for v in var]
        self._user_vars = var
        self.len_ = len(self.vars)
        self.u_model = TanhMLP(self.layer_sizes, device=self.device)
        if ctx.is_distributed:
            ctx.broadcast_(self.u_model.flat.data)
        self.tf_optimizer = Adam(lr=0.005, beta_1=0.99)
        self.tf_optimizer_vars = Adam(lr=0.005, beta_1=0.99)
        self.tf_optimizer_weights = Adam(lr=0.005, beta_1=0.99)
        if col_weights is not None:
            cw = torch.as_tensor(col_weights.detach().cpu().numpy() if torch.is_tensor(col_weights)
                                 else np.asarray(col_weights), dtype=torch.float32).reshape(-1, 1)
            if ctx.is_distributed:
                cw = cw.to(self.device)
                ctx.broadcast_(cw)
            self.col_weights = cw[self._lo:self._hi].to(self.device).contiguous().detach().requires_grad_(True)
        else:
            self.col_weights = None
        self.backend = backend
        self.precision = precision
        self.newton_precision = newton_precision
        from ..config import DEFAULT_LBFGS_STOP
        self.lbfgs_stop = lbfgs_stop or DEFAULT_LBFGS_STOP
        self._engine = None
        self._program = None
        self._programs = {}
        self._engines = {}
        self._state = None
        self.fit_info = {}

    # ------------------------------------------------------------------ program ----------
    def program(self, precision=None):
        """Loss program (Adam precision, or ``precision`` for the L-BFGS objective)."""
        if precision is not None and precision != self.precision:
            prog = self._programs.get(precision)
            if prog is None or prog.net is not self.u_model:
                prog = self._programs[precision] = self._build_program(precision)
                self._engines.pop(precision, None)
            return prog
        if self._program is None or self._program.net is not self.u_model:
            self._program = self._build_program(self.precision)
            self._engine = None
        return self._program

    def _build_program(self, precision):
        ctx = self.dist_ctx
        world = ctx.world if ctx.is_distributed else 1
        g = (lambda l: l * l) if self.col_weights is not None else None
        prog = LossProgram(self.u_model, self.X.shape[1], self.device, backend=self.backend,
                           precision=precision, world=world, g=g)
        s = prog.add_segment("data", self.X)
        prog.register_callable(self.f_model, s, extra_args=(self.vars,))
        denom = float(self.N) if world > 1 else None
        prog.add_term(Term("Data", "data", seg=s, val=self.u, denom=denom))
        prog.add_term(Term("Residual_0", "residual", seg=s, fn=self.f_model, extra=(self.vars,),
                           index=0, lam=0 if self.col_weights is not None else None, denom=denom))
        prog.finalize()
        prog.enable_fusion(self._lambdas(), extras=(self.vars,))
        return prog

    def _lambdas(self):
        return [self.col_weights] if self.col_weights is not None else []

    def _train_state(self, device):
        if self._state is None:
            flat = self.u_model.flat
            self._state = {"best_loss": torch.full((), float("inf"), device=device),
                           "best_flat": flat.detach().clone(),
                           "best_epoch": torch.full((), -1, dtype=torch.int64, device=device),
                           "epoch": torch.zeros((), dtype=torch.int64, device=device),
                           "epoch_host": 0, "hist": None}
        return self._state

    def loss(self):
        total, _ = self.program().evaluate(self.u_model.flat, self._lambdas())
        return total

    def grad(self):
        loss = self.loss()
        wrt = [self.u_model.flat] + self._lambdas() + self.vars
        grads = torch.autograd.grad(loss, wrt, allow_unused=True)
        return loss, [torch.zeros_like(w) if g is None else g for g, w in zip(grads, wrt)]

    @property
    def variables(self):
        return [self.u_model.flat] + self._lambdas() + self.vars

    def _get_engine(self, n_hint, precision=None):
        if precision is not None and precision != self.precision:
            prog = self.program(precision)
            eng = self._engines.get(precision)
            if eng is None or eng.program is not prog:
                eng = self._engines[precision] = self._new_engine(prog, n_hint)
            return eng
        prog = self.program()
        if self._engine is None or self._engine.program is not prog:
            self._engine = self._new_engine(prog, n_hint)
        return self._engine

    def _new_engine(self, prog, n_hint):
        rep = not self.dist_ctx.is_distributed
        groups = [ParamGroup([self.u_model.flat], lambda: self.tf_optimizer, 1.0),
                  ParamGroup(self._lambdas(), lambda: self.tf_optimizer_weights, -1.0, [rep]),
                  ParamGroup(self.vars, lambda: self.tf_optimizer_vars, 1.0)]
        ncw = len(self._lambdas())

        def bind(alias):
            return {"params": alias[0], "lambdas": alias[1:1 + ncw], "extras": (alias[1 + ncw:],)}
        return AdamEngine(self, prog, groups, n_steps_hint=n_hint, lambdas=self._lambdas(), bind=bind)

    def train_op(self):
        return self._get_engine(1).run(1)

    def fit(self, tf_iter=0, newton_iter=0):
        """Adam for ``tf_iter`` steps (reference ``fit``, models.py:381-396), then L-BFGS over the
        network and the coefficients for ``newton_iter`` iterations."""
        import time
        from ..profiling import maybe_profile
        with maybe_profile(f"DiscoveryModel.fit(tf_iter={tf_iter}, newton_iter={newton_iter})"):
            if tf_iter > 0:
                t0 = time.perf_counter()
                self.train_loop(tf_iter)
                self.fit_info["adam"] = {"steps": int(tf_iter), "wall_s": time.perf_counter() - t0}
            if newton_iter > 0:
                t0 = time.perf_counter()
                info = self._fit_lbfgs(int(newton_iter))
                info["wall_s"] = time.perf_counter() - t0
                self.fit_info["lbfgs"] = info

    def _fit_lbfgs(self, newton_iter):
        """Device L-BFGS (the collocation solver's, optimizers/lbfgs_device.py) on
        ``x = [theta | coefficients]``: every evaluation writes ``x`` into the network buffer and the
        coefficient tensors, then one fused loss + gradient pass (the Adam engine's phase A, whose
        fused loss already emits the coefficient gradients) fills ``[grad theta | grad c | loss]``."""
        from ..fit import _use_graphs
        from ..optimizers import lbfgs, lbfgs_device
        ctx = self.dist_ctx
        eng = self._get_engine(1, self.newton_precision)
        flat = self.u_model.flat
        P = flat.numel()
        sizes = [v.numel() for v in self.vars]
        ncw = len(self._lambdas())
        var_idx = [1 + ncw + k for k in range(len(self.vars))]
        x = torch.cat([flat.detach().reshape(-1)] + [v.detach().reshape(-1) for v in self.vars]).contiguous()
        fg = torch.empty(x.numel() + 1, dtype=torch.float32, device=self.device)

        def load_x(src):
            with torch.no_grad():
                flat.copy_(src[:P])
                off = P
                for v, n in zip(self.vars, sizes):
                    v.view(-1).copy_(src[off:off + n])
                    off += n

        def evaluate():
            load_x(x)
            total, grads, _ = eng._phase_a(for_step=False)
            torch.cat([grads[0].reshape(-1)] + [grads[i].reshape(-1) for i in var_idx] + [total.reshape(1)], out=fg)
            return fg

        if self.verbose and ctx.rank == 0:
            print("Starting L-BFGS training (network + coefficients)")
        if self.device.type == "cuda":
            opt = lbfgs_device.minimize(evaluate, x, newton_iter, lr=0.8,
                                        all_reduce=ctx.all_reduce_ if ctx.is_distributed else None,
                                        capture_all_reduce=ctx.capturable(x.numel() + 1),
                                        use_graph=_use_graphs(self.device), stop=self.lbfgs_stop)
            ctx.check_health()
            load_x(opt.best_x)
            info = {"impl": "device", "n_iter": opt.n_iter, "reason": opt.reason, "min_loss": opt.min_loss}
        else:
            def loss_and_grad(w):
                x.copy_(w)
                buf = evaluate().clone()
                if ctx.is_distributed:
                    ctx.all_reduce_(buf)
                return buf[-1], buf[:-1]
            state = lbfgs.Struct()
            _, _, _, best_w, min_loss, _ = lbfgs.eager_lbfgs(loss_and_grad, x.clone(), state=state, maxIter=newton_iter,
                                                           learningRate=0.8, stop=self.lbfgs_stop)
            load_x(best_w)
            info = {"impl": "host", "n_iter": int(getattr(state, "nIter", 0)), "reason": getattr(state, "reason", "?"),
                    "min_loss": float(min_loss)}
        self._sync_user_vars()
        # (step, values) like the Adam entries: the step count after the L-BFGS iterations
        last = self.var_history[-1][0] if self.var_history else 0
        self.var_history.append((int(last) + int(info["n_iter"]), [float(v.detach()) for v in self.vars]))
        info["var_history_index"] = len(self.var_history) - 1
        if self.verbose and ctx.rank == 0:
            print(f"L-BFGS stopped after {info['n_iter']} iterations: {info['reason']}")
        return info

    def train_loop(self, tf_iter):
        ctx = self.dist_ctx
        if self.verbose and ctx.rank == 0:
            print_screen(self, discovery_model=True)
        eng = self._get_engine(tf_iter)
        bar = tqdm(total=tf_iter, disable=not (self.verbose and ctx.rank == 0), desc="Adam")

        def progress(done, loss):
            bar.n = done
            vals = [float(v.detach()) for v in self.vars]
            self.var_history.append((done, vals))
            if loss is not None:
                bar.set_postfix(loss=loss, vars=vals)
            bar.refresh()

        eng.run(tf_iter, progress=progress, log_every=self.log_every)
        bar.close()
        self._sync_user_vars()

    def _sync_user_vars(self):
        """Mirror learned coefficients into user-supplied tensors (tf.Variable semantics)."""
        with torch.no_grad():
            for uv, v in zip(self._user_vars, self.vars):
                if torch.is_tensor(uv) and uv is not v and uv.numel() == v.numel():
                    uv.copy_(v.detach().to(uv.device))

    def predict(self, X_star, chunk=65536):
        X = torch.as_tensor(np.asarray(X_star), dtype=torch.float32, device=self.device)
        with torch.no_grad():
            u = torch.cat([self.u_model(X[i:i + chunk]) for i in range(0, X.shape[0], chunk)])
        f = self.program().residual_on(self.f_model, X, extra=(self.vars,), chunk=chunk)
        return u.cpu().numpy(), f[0].cpu().numpy()
