"""``DiscoveryModel`` - inverse problems: learn PDE coefficients from observations.

Reference: tensordiffeq/models.py:324-396.  ``compile(layer_sizes, f_model, X, u, var,
col_weights=None)`` with ``f_model(u_model, var, *X)``; loss ``MSE(u(X), u*) + MSE(f, 0)`` or,
with self-adaptive collocation weights, ``MSE(u(X), u*) + mean(col_weights^2 f^2)``; three Adam
instances (network, coefficients, weights - the weights by gradient ascent).

Fixed: the reference never updated the last output bias (``grads[:-(len_+2)]`` truncation,
B22) - every parameter trains here.  The observation points are served by the same single jet
evaluation as the residual (one HIP jet pass covers u and every derivative the residual needs),
and data parallelism shards the observations.
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
                backend="auto", device=None, seed=None, precision=None):
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
        self._engine = None
        self._program = None
        self._state = None

    # ------------------------------------------------------------------ program ----------
    def program(self):
        if self._program is None or self._program.net is not self.u_model:
            ctx = self.dist_ctx
            world = ctx.world if ctx.is_distributed else 1
            g = (lambda l: l * l) if self.col_weights is not None else None
            prog = LossProgram(self.u_model, self.X.shape[1], self.device, backend=self.backend,
                           precision=self.precision,
                               world=world, g=g)
            s = prog.add_segment("data", self.X)
            prog.register_callable(self.f_model, s, extra_args=(self.vars,))
            denom = float(self.N) if world > 1 else None
            prog.add_term(Term("Data", "data", seg=s, val=self.u, denom=denom))
            prog.add_term(Term("Residual_0", "residual", seg=s, fn=self.f_model, extra=(self.vars,),
                               index=0, lam=0 if self.col_weights is not None else None, denom=denom))
            prog.finalize()
            prog.enable_fusion(self._lambdas(), extras=(self.vars,))
            self._program = prog
            self._engine = None
        return self._program

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

    def _get_engine(self, n_hint):
        prog = self.program()
        if self._engine is None:
            rep = not self.dist_ctx.is_distributed
            groups = [ParamGroup([self.u_model.flat], lambda: self.tf_optimizer, 1.0),
                      ParamGroup(self._lambdas(), lambda: self.tf_optimizer_weights, -1.0, [rep]),
                      ParamGroup(self.vars, lambda: self.tf_optimizer_vars, 1.0)]
            ncw = len(self._lambdas())

            def bind(alias):
                return {"params": alias[0], "lambdas": alias[1:1 + ncw], "extras": (alias[1 + ncw:],)}
            self._engine = AdamEngine(self, prog, groups, n_steps_hint=n_hint, lambdas=self._lambdas(),
                                      bind=bind)
        return self._engine

    def train_op(self):
        return self._get_engine(1).run(1)

    def fit(self, tf_iter):
        from ..profiling import maybe_profile
        with maybe_profile(f"DiscoveryModel.fit(tf_iter={tf_iter})"):
            self.train_loop(tf_iter)

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
