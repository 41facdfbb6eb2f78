"""``CollocationSolverND`` - forward collocation PINN solver.

Reference: tensordiffeq/models.py:12-319.  Same public surface: ``compile(layer_sizes, f_model,
domain, bcs, Adaptive_type=0, dict_adaptive=None, init_weights=None, g=None, dist=False)``,
``compile_data``, ``update_loss``, ``grad``, ``fit(tf_iter, newton_iter, batch_sz,
newton_eager)``, ``get_loss_and_flat_grad``, ``predict(X_star, best_model=False)``, ``save``,
``load_model``; attributes ``u_model``, ``tf_optimizer``, ``tf_optimizer_weights`` (replaceable),
``lambdas``, ``lambdas_map``, ``losses``, ``min_loss``, ``best_epoch``, ``best_model``.

Implements the reference's *intent* where it is broken: ``Adaptive_type`` accepts
ints and names (B14); SA works with minibatches and under DP (B5); DP shards points (B3) and
reports the true global loss (B4); repeated ``fit`` calls resume (B6); L-BFGS runs under DP
(B7); best weights are real snapshots (B8); the data-assimilation term is used (B17).
"""
from __future__ import annotations

import math
import os
import time

import numpy as np
import torch
from tqdm.auto import tqdm

from .. import checkpoint
from ..fit import AdamEngine, LossGradEngine, ParamGroup
from ..optimizers import Adam, eager_lbfgs
from ..output import print_screen
from ..parallel import dist as pdist
from .loss import LossProgram, Term
from .networks import FlatModule, TanhMLP

_ADAPTIVE = {0: 0, "none": 0, "baseline": 0, "pinn": 0,
             1: 1, "self-adaptive": 1, "self_adaptive": 1, "sa": 1, "sa-pinn": 1,
             2: 2, "loss-weights": 2, "self-adaptive-loss": 2, "weight_outside_sum": 2,
             3: 3, "ntk": 3}


def parse_adaptive_type(a):
    key = a.lower() if isinstance(a, str) else a
    if key not in _ADAPTIVE:
        raise Exception("Adaptive method invalid!")
    v = _ADAPTIVE[key]
    if v == 3:
        raise NotImplementedError("NTK adaptive weighting (Adaptive_type=3) is not implemented")
    return v


def default_device():
    ctx = pdist._CTX
    if ctx is not None:
        return ctx.device
    return torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")


class _FlatModel:
    """Callable view of the network evaluated at a frozen flat snapshot (``best_model`` values)."""

    def __init__(self, net, flat):
        self.net, self.flat = net, flat

    def __call__(self, *xs):
        with torch.no_grad():
            return self.net(*xs, params=self.flat)


class CollocationSolverND:
    def __init__(self, assimilate=False, verbose=True):
        self.assimilate = assimilate
        self.verbose = verbose
        self.best_epoch = {"adam": -1, "l-bfgs": -1, "overall": -1}
        self.min_loss = {"adam": np.inf, "l-bfgs": np.inf, "overall": np.inf}
        self.best_model = {"adam": None, "l-bfgs": None, "overall": None}
        self.lambdas = self.dict_adaptive = self.lambdas_map = None
        self.data_x = self.data_t = self.data_s = None
        self._engine = None
        self._lbfgs_engine = None
        self._state = None
        self._programs = {}
        self._best_flat = {}
        self.fit_info = {}    # last fit(): per-phase steps / wall time, L-BFGS stop reason
        self.log_every = 100
        self.metrics = None   # MetricsLogger (compile(metrics_path=...) or TDQ_METRICS)

    # ================================================================== compile =========
    def compile(self, layer_sizes, f_model, domain, bcs, Adaptive_type=0, dict_adaptive=None,
                init_weights=None, g=None, dist=False, backend="auto", device=None,
                periodic_legacy=False, seed=None, network=None, precision=None, metrics_path=None,
                log_every=None, newton_precision=None, lbfgs_stop=None, newton_schedule=None):
        from ..config import SolverConfig
        self.config = SolverConfig.from_env(backend=None if backend == "auto" else backend, precision=precision,
                                            seed=seed, metrics_path=metrics_path, log_every=log_every,
                                            newton_precision=newton_precision, lbfgs_stop=lbfgs_stop,
                                            newton_schedule=newton_schedule)
        backend = self.config.backend
        precision = self.config.precision
        # jet-GEMM precision of the L-BFGS phase (None: same as the Adam phase).  L-BFGS's
        # curvature pairs need the accurate gradient; Adam tolerates bf16 activations
        # (profiles/r2_v2_accuracy_mixed.jsonl)
        self.newton_precision = self.config.newton_precision
        # leading L-BFGS phases in other precisions, e.g. [("bf16", 7000)]: cheaper iterations first,
        # the newton_precision phase (fresh history from the best iterate) polishes
        from ..config import parse_newton_schedule
        self.newton_schedule = parse_newton_schedule(self.config.newton_schedule)
        if precision == "bf16" and (self.newton_precision or precision) == "bf16":
            from .loss import _warn_once
            _warn_once("precision='bf16' also for L-BFGS: its curvature pairs need accurate gradients (AC-SA "
                       "stalls at L2 6-7e-2 vs 2.2e-2 with newton_precision='bf16x3'), and residuals dominated by "
                       "second derivatives with large sources lose accuracy in bf16 (Helmholtz L2 9.4e-2 vs 7.9e-3 "
                       "in bf16x3); consider newton_precision='bf16x3' or precision='bf16x3'")
        seed = self.config.seed
        periodic_legacy = periodic_legacy or self.config.periodic_legacy
        self.log_every = self.config.log_every
        if seed is not None:
            from ..utils.seeding import set_seed
            set_seed(seed)
        self.dist = bool(dist)
        self.dist_ctx = pdist.init_distributed(auto_launch=True) if dist else pdist.get_context(device)
        self.device = torch.device(device) if device is not None else (
            self.dist_ctx.device if dist else default_device())
        self.tf_optimizer = Adam(lr=0.005, beta_1=0.99)
        self.tf_optimizer_weights = Adam(lr=0.005, beta_1=0.99)
        self.layer_sizes = list(layer_sizes)
        self.sizes_w = [layer_sizes[i] * layer_sizes[i - 1] for i in range(1, len(layer_sizes))]
        self.sizes_b = list(layer_sizes[1:])
        self.bcs = list(bcs)
        self.f_model = f_model
        self.g = g
        self.domain = domain
        self.backend = backend
        self.precision = precision
        self.periodic_legacy = periodic_legacy
        if domain.X_f is None:
            raise ValueError("call domain.generate_collocation_points(N_f) before compile")
        X_f = torch.as_tensor(np.asarray(domain.X_f) if not torch.is_tensor(domain.X_f) else domain.X_f,
                              dtype=torch.float32)
        self.N_f = int(X_f.shape[0])
        if self.config.metrics_path:
            from ..metrics import MetricsLogger
            self.metrics = MetricsLogger(self.config.metrics_path, self.dist_ctx.rank, self.dist_ctx.world,
                                         n_points=None)
        ctx = self.dist_ctx
        self._lo, self._hi = pdist.shard_range(self.N_f, ctx.rank, ctx.world)
        self.X_f_local = X_f[self._lo:self._hi].to(self.device)
        self.X_f_in = [self.X_f_local[:, j:j + 1] for j in range(X_f.shape[1])]
        self.X_f_len = np.array([self.N_f])
        if network is not None and not isinstance(network, (TanhMLP, FlatModule)):
            network = FlatModule(network)
        self.u_model = network if network is not None else TanhMLP(self.layer_sizes, device=self.device)
        self.u_model.to(self.device)
        if ctx.is_distributed:
            ctx.broadcast_(self.u_model.flat.data)

        self.Adaptive_type = parse_adaptive_type(Adaptive_type)
        self.isAdaptive = self.Adaptive_type in (1, 2)
        self.weight_outside_sum = self.Adaptive_type == 2
        if not self.isAdaptive and dict_adaptive is not None and init_weights is not None:
            raise Exception("Adaptive weights are turned off but weight vectors were provided. "
                            "Set the weight vectors to \"none\" to continue")
        if self.isAdaptive:
            if dict_adaptive is None or init_weights is None:
                raise Exception("Adaptive weights selected but no inputs were specified!")
            if all(not any(v) for v in dict_adaptive.values()):
                raise Exception("Adaptive method was selected but none loss was marked to be adaptive")
            self.dict_adaptive = dict_adaptive
            self._init_lambdas(init_weights, dict_adaptive)
        else:
            self.lambdas, self.lambdas_map, self._lam_kind = [], {"residual": [], "bcs": []}, []
            self._lam_for = {}
        self._programs = {}
        self._engine = None
        self._lbfgs_engine = None
        self._state = None

    def _init_lambdas(self, init_weights, dict_adaptive):
        ctx = self.dist_ctx
        lambdas, lmap, kinds, lam_for = [], {}, [], {}
        for key in ("residual", "BCs"):
            vals = init_weights.get(key, init_weights.get(key.lower(), []))
            flags = dict_adaptive.get(key, dict_adaptive.get(key.lower(), []))
            idx = []
            for j, value in enumerate(vals):
                if value is None or not (j < len(flags) and flags[j]):
                    continue
                t = torch.as_tensor(value.detach().cpu().numpy() if torch.is_tensor(value) else np.asarray(value),
                                    dtype=torch.float32).to(self.device)
                if ctx.is_distributed:
                    ctx.broadcast_(t)
                # per-point residual weights are sharded with the points - except under
                # Adaptive_type 2 ("outside sum": (sum_i w_i) * mean(r^2), reference utils.py:38-44),
                # whose sum over ALL weights multiplies every rank's partial mean: those weights stay
                # replicated and their gradient (the global mean) is all-reduced like theta's
                sharded = (key == "residual" and t.numel() == self.N_f and ctx.is_distributed
                           and not self._outside_sum_weights())
                if sharded:
                    t = t.reshape(-1, 1)[self._lo:self._hi]
                t = t.reshape(-1, 1).contiguous() if t.numel() > 1 else t.reshape(()).contiguous()
                lambdas.append(t.detach().requires_grad_(True))
                kinds.append("residual" if key == "residual" else "bc")
                idx.append(len(lambdas) - 1)
                lam_for[(kinds[-1], j)] = len(lambdas) - 1
            lmap[key.lower()] = idx
        self.lambdas, self.lambdas_map, self._lam_kind = lambdas, lmap, kinds
        self._lam_for = lam_for

    def compile_data(self, x, t, y):
        if not self.assimilate:
            raise Exception("Assimilate needs to be set to 'true' for data assimilation. Re-initialize "
                            "CollocationSolverND with assimilate=True.")
        self.data_x, self.data_t, self.data_s = x, t, y
        self._programs = {}
        self._engine = None

    # ================================================================== program =========
    def _adaptive_flags(self, key):
        if not self.isAdaptive:
            return []
        d = self.dict_adaptive
        return list(d.get(key, d.get(key.lower(), [])))

    def _residual_count(self):
        from .loss import _Float64View
        is_mlp = isinstance(self.u_model, TanhMLP)
        probe = self.X_f_local[:4].detach()
        probe = probe.double() if is_mlp else probe
        cols = [probe[:, j:j + 1].clone().requires_grad_(True) for j in range(probe.shape[1])]
        net = _Float64View(self.u_model) if is_mlp else self.u_model
        out = self.f_model(net, *cols)
        return len(out) if isinstance(out, (tuple, list)) else 1

    def _build_program(self, batch=None, precision=None):
        ctx = self.dist_ctx
        world = ctx.world if ctx.is_distributed else 1
        rep_scale = 1.0 / world
        prog = LossProgram(self.u_model, len(self.domain.vars), self.device, backend=self.backend,
                           precision=precision or self.precision,
                           world=world, weight_outside_sum=self.weight_outside_sum, g=self.g,
                           periodic_legacy=self.periodic_legacy)
        for i, bc in enumerate(self.bcs):
            lam = self._lam_for.get(("bc", i))
            name = f"BC_{i}"
            if bc.isPeriodic:
                pairs = []
                for k in range(len(bc.upper_points)):
                    su = prog.add_segment(f"{name}_up{k}", bc.upper_points[k])
                    sl = prog.add_segment(f"{name}_lo{k}", bc.lower_points[k])
                    pairs.append((su, sl))
                    for fn in bc.deriv_model:
                        prog.register_callable(fn, su)
                        prog.register_callable(fn, sl)
                prog.add_term(Term(name, "periodic", pairs=pairs, fns=list(bc.deriv_model), lam=lam,
                                   scale=rep_scale))
            elif bc.isNeumann:
                segs = []
                for k, pts in enumerate(bc.points):
                    s = prog.add_segment(f"{name}_n{k}", pts)
                    segs.append(s)
                    for fn in bc.deriv_model:
                        prog.register_callable(fn, s)
                val = torch.as_tensor(np.asarray(bc.val), dtype=torch.float32, device=self.device).reshape(-1, 1)
                prog.add_term(Term(name, "neumann", segs=segs, fns=list(bc.deriv_model), val=val,
                                   lam=lam, scale=rep_scale))
            elif bc.isInit or bc.isDirichlect:
                s = prog.add_segment(name, bc.input)
                val = bc.val
                val = torch.as_tensor(np.asarray(val) if not torch.is_tensor(val) else val.detach().cpu(),
                                      dtype=torch.float32, device=self.device)
                val = val.reshape(-1, 1) if val.numel() > 1 else val.reshape(())
                prog.add_term(Term(name, "ic" if bc.isInit else "dirichlet", seg=s, val=val, lam=lam,
                                   scale=rep_scale))
            else:
                raise Exception("Boundary condition type is not acceptable")
        if self.assimilate and self.data_s is not None:
            Xd = np.hstack([np.reshape(np.asarray(self.data_x), (-1, 1)),
                            np.reshape(np.asarray(self.data_t), (-1, 1))])
            s = prog.add_segment("data", Xd)
            val = torch.as_tensor(np.reshape(np.asarray(self.data_s), (-1, 1)), dtype=torch.float32,
                                  device=self.device)
            prog.add_term(Term("Data", "data", seg=s, val=val, scale=rep_scale))
        Xr = self.X_f_local
        n_glob = self.N_f
        if batch is not None:
            lo, hi = batch
            Xr = Xr[lo:hi]
            n_glob = (hi - lo) * world
        sr = prog.add_segment("residual", Xr)
        prog.register_callable(self.f_model, sr)
        n_res = self._n_res if hasattr(self, "_n_res") else self._residual_count()
        self._n_res = n_res
        for k in range(n_res):
            lam = self._lam_for.get(("residual", k))
            term = Term(f"Residual_{k}", "residual", seg=sr, fn=self.f_model, extra=(), index=k,
                        lam=lam, denom=float(n_glob) if world > 1 or batch is not None else None)
            if batch is not None and lam is not None and self.lambdas[lam].numel() > 1:
                term.lam_range = batch
            prog.add_term(term)
        prog.finalize()
        return prog

    def program(self, batch=None, precision=None):
        self._flat()  # wraps a user-assigned custom network
        if self._state is not None:
            self._train_state(self.device)  # re-validates the best snapshot against the network
        if self._programs.get("net") is not self.u_model:
            self._programs = {"net": self.u_model}
            self._engine = None
            self._lbfgs_engine = None
        if precision == self.precision:
            precision = None
        key = ("batch", batch) if precision is None else ("batch", batch, precision)
        if key not in self._programs:
            prog = self._build_program(batch, precision)
            prog.enable_fusion(self.lambdas)
            self._programs[key] = prog
        return self._programs[key]

    @property
    def active_backend(self):
        return self.program().backend

    # ================================================================== state ===========
    def _train_state(self, device):
        flat = self._flat()
        st = self._state
        if st is not None and (st["best_flat"].numel() != flat.numel() or st["best_flat"].device != flat.device):
            # the network was replaced (load_model with other layer sizes, a custom u_model): the
            # best-weights snapshot belongs to the old parameter vector - restart best tracking
            # (epoch counter and loss history are kept); compiled engines are dropped with it
            st["best_flat"] = flat.detach().clone()
            st["best_loss"] = torch.full((), math.inf, dtype=torch.float32, device=flat.device)
            st["best_epoch"] = torch.full((), -1, dtype=torch.int64, device=flat.device)
            st.pop("improved", None)
            self._programs = {}
            self._engine = None
            self._lbfgs_engine = None
        if self._state is None:
            self._state = {
                "best_loss": torch.full((), math.inf, dtype=torch.float32, device=device),
                "best_flat": flat.detach().clone(),
                "best_epoch": torch.full((), -1, dtype=torch.int64, device=device),
                "epoch": torch.zeros((), dtype=torch.int64, device=device),
                "epoch_host": 0,
                "hist": None,
            }
        return self._state

    def _flat(self):
        if not isinstance(self.u_model, (TanhMLP, FlatModule)):
            self.u_model = FlatModule(self.u_model).to(self.device)  # user replaced u_model
        return self.u_model.flat

    @property
    def variables(self):
        return [self._flat()] + list(self.lambdas or [])

    def _outside_sum_weights(self):
        """Per-point residual weights enter through MSE's outside sum (Adaptive_type 2 without
        ``g``): their sum over ALL points multiplies every rank's partial mean, so under DP they stay
        replicated.  With ``g`` the residual term is g_MSE, element-wise g(lam) * f^2 (reference
        utils.py:47-48), and the weights are sharded with their points like type 1's."""
        return self.weight_outside_sum and self.g is None

    def _lam_replicated(self):
        ctx = self.dist_ctx
        return [not (k == "residual" and ctx.is_distributed and l.numel() > 1 and not self._outside_sum_weights())
                for l, k in zip(self.lambdas, self._lam_kind)]

    # ================================================================== loss API =========
    def update_loss(self):
        total, vals = self.program().evaluate(self._flat(), self.lambdas)
        self.loss_terms = {k: v.detach() for k, v in vals.items()}
        return total

    def grad(self):
        loss = self.update_loss()
        grads = torch.autograd.grad(loss, self.variables, allow_unused=True)
        return loss, [torch.zeros_like(v) if g is None else g for g, v in zip(grads, self.variables)]

    def get_loss_and_flat_grad(self):
        eng = self._get_lbfgs_engine()
        return lambda w: eng(torch.as_tensor(w, dtype=torch.float32, device=self.device))

    def _get_lbfgs_engine(self, precision=None):
        """The L-BFGS objective's engine at ``precision`` (default ``newton_precision``)."""
        default = self.newton_precision or self.precision
        prec = precision or default
        if prec != default:
            key = ("lbfgs_engine", prec)
            eng = self._programs.get(key)
            prog = self.program(precision=prec)
            if eng is None or eng.program is not prog:
                eng = self._programs[key] = LossGradEngine(self, prog, self.lambdas)
            return eng
        if self._lbfgs_engine is None:
            self._lbfgs_engine = LossGradEngine(self, self.program(precision=prec), self.lambdas)
        return self._lbfgs_engine

    def _get_engine(self, batch=None, n_hint=0):
        key = ("engine", batch)
        eng = self._programs.get(key)
        prog = self.program(batch)
        if eng is None:
            groups = [ParamGroup([self._flat()], lambda: self.tf_optimizer, 1.0),
                      ParamGroup(self.lambdas, lambda: self.tf_optimizer_weights, -1.0,
                                 self._lam_replicated())]
            eng = AdamEngine(self, prog, groups, n_steps_hint=n_hint, lambdas=self.lambdas)
            self._programs[key] = eng
        return eng

    # ================================================================== fit =============
    def minibatches(self, batch_sz):
        """Per-rank minibatch ranges ``[(lo, hi), ...]`` (local shard indices) or ``[None]`` for
        full batch.  The count comes from the SMALLEST shard (``N_f // world``), so every rank
        runs the same number of steps - and therefore the same number of collectives - per
        epoch even when ``N_f`` does not divide evenly; each step's residual denominator is
        ``batch_sz * world`` on every rank."""
        if batch_sz is None:
            return [None]
        batch_sz = int(batch_sz)
        if batch_sz <= 0:
            raise ValueError(f"batch_sz must be positive, got {batch_sz}")
        ctx = self.dist_ctx
        world = ctx.world if ctx.is_distributed else 1
        n_min = self.N_f // world
        if batch_sz >= n_min:
            return [None]
        nb = n_min // batch_sz
        return [(i * batch_sz, (i + 1) * batch_sz) for i in range(nb)]

    def fit(self, tf_iter=0, newton_iter=0, batch_sz=None, newton_eager=True):
        from ..profiling import maybe_profile
        with maybe_profile(f"CollocationSolverND.fit(tf_iter={tf_iter}, newton_iter={newton_iter})"):
            return self._fit(tf_iter, newton_iter, batch_sz, newton_eager)

    def _fit(self, tf_iter, newton_iter, batch_sz, newton_eager):
        ctx = self.dist_ctx
        batches = self.minibatches(batch_sz)
        if self.verbose and ctx.rank == 0:
            print_screen(self)
        self.program()  # build / plan before timing-sensitive loops
        start_epoch = self._train_state(self.device)["epoch_host"]
        if tf_iter > 0:
            if self.verbose and ctx.rank == 0:
                print("Starting Adam training")
            bar = tqdm(total=tf_iter, disable=not (self.verbose and ctx.rank == 0), desc="Adam")

            if self.metrics is not None:
                self.metrics.n_points = self.X_f_local.shape[0]
                self.metrics.mark(start_epoch)
                if ctx.is_distributed:  # which collective carries the DP bucket (and its start-up timing)
                    self.metrics.log_event("allreduce", world=ctx.world, **ctx.allreduce_info)

            def progress(done, loss):
                bar.n = done
                if loss is not None:
                    bar.set_postfix(loss=loss)
                    if self.metrics is not None:
                        self._log_metrics("adam", loss)
                bar.refresh()

            t_adam = time.perf_counter()
            self._prebuild_lbfgs_objective()
            if batches == [None]:
                eng = self._get_engine(None, tf_iter)
                eng.run(tf_iter, progress=progress, log_every=self.log_every)
            else:
                engines = [self._get_engine(b, tf_iter * len(batches)) for b in batches]
                for ep in range(tf_iter):
                    for eng in engines:
                        loss = eng.run(1, use_graph=False)
                    if (ep + 1) % self.log_every == 0 or ep + 1 == tf_iter:
                        progress(ep + 1, float(loss))
            bar.close()
            st = self._state
            self.min_loss["adam"] = float(st["best_loss"])   # (device sync: the phase is done)
            self.fit_info["adam"] = {"steps": int(tf_iter), "wall_s": time.perf_counter() - t_adam}
            self.best_epoch["adam"] = int(st["best_epoch"])
            self._best_flat["adam"] = st["best_flat"].clone()
            self.best_model["adam"] = _FlatModel(self.u_model, self._best_flat["adam"])
        if newton_iter > 0:
            self._fit_lbfgs(newton_iter, newton_eager)
        self._select_overall(start_epoch, tf_iter)

    def _log_metrics(self, phase, loss):
        st = self._state
        ep = int(st["epoch_host"])
        terms = None
        if st["hist"] is not None and ep > 0:
            row = st["hist"][ep - 1].detach().cpu().tolist()
            terms = {t.name: v for t, v in zip(self.program().terms, row[1:])}
        self.metrics.log(phase, ep, loss, terms)

    def _use_device_lbfgs(self):
        """Device-resident L-BFGS (``optimizers/lbfgs_device.py``) by default on a GPU; the
        host-driven port elsewhere.  ``TDQ_LBFGS`` / ``SolverConfig.lbfgs`` overrides."""
        impl = getattr(getattr(self, "config", None), "lbfgs", "auto")
        if impl == "auto":
            return self.device.type == "cuda"
        return impl == "device"

    def _prebuild_lbfgs_objective(self):
        """Start the hipRTC compile of the L-BFGS objective's one-launch kernel (ops/fused_step.py
        ``prebuild``) on a host thread, so it overlaps the Adam phase instead of opening the
        L-BFGS phase (~0.35 s for the bf16x3 objective).  Timed inside the Adam phase."""
        if self.device.type != "cuda" or os.environ.get("TDQ_PREBUILD", "1") == "0":
            return
        try:
            from ..ops import fused_step
            prog = self.program(precision=self.newton_precision or self.precision)
            if prog.backend == "hip":
                fused_step.prebuild(prog)
        except Exception:  # noqa: BLE001 - an optimisation only: the L-BFGS phase compiles it itself
            pass

    def _fit_lbfgs(self, newton_iter, newton_eager):
        t0 = time.perf_counter()
        info = self._fit_lbfgs_body(newton_iter, newton_eager)
        info["wall_s"] = time.perf_counter() - t0
        info["max_iter"] = int(newton_iter)
        self.fit_info["lbfgs"] = info
        if self.metrics is not None:
            self.metrics.log_event("lbfgs_stop", **info)
        if self.verbose and self.dist_ctx.rank == 0:
            print(f"L-BFGS stopped after {info['n_iter']} iterations: {info['reason']}")

    def _fit_lbfgs_body(self, newton_iter, newton_eager):
        """Run L-BFGS; returns ``{"impl", "n_iter", "func_evals", "reason", "stop"}``.  With a
        ``newton_schedule`` the leading phases run first (each from the previous phase's best
        iterate, device L-BFGS only), then the ``newton_precision`` phase takes the rest."""
        sched = list(getattr(self, "newton_schedule", None) or [])
        if sched and newton_eager and self._use_device_lbfgs():
            phases = []
            left = int(newton_iter)
            for prec, n in sched:
                n = min(n, left)
                if n <= 0:
                    break
                info = self._fit_lbfgs_phase(n, self._get_lbfgs_engine(prec))
                phases.append({"precision": prec, **{k: info[k] for k in ("n_iter", "reason")}})
                left -= n
            if left > 0:
                info = self._fit_lbfgs_phase(left, self._get_lbfgs_engine())
                phases.append({"precision": self.newton_precision or self.precision,
                               **{k: info[k] for k in ("n_iter", "reason")}})
            info = dict(info)
            info["n_iter"] = sum(p["n_iter"] for p in phases)
            info["phases"] = phases
            return info
        if sched:
            from .loss import _warn_once
            _warn_once("newton_schedule is honoured by the device L-BFGS only (newton_eager=True on a GPU, "
                       "TDQ_LBFGS=device); this L-BFGS path runs one phase at newton_precision")
        return self._fit_lbfgs_phase(newton_iter, None, newton_eager)

    def _fit_lbfgs_phase(self, newton_iter, eng=None, newton_eager=True):
        ctx = self.dist_ctx
        stop = getattr(getattr(self, "config", None), "lbfgs_stop", "legacy")
        if self.verbose and ctx.rank == 0:
            print("Starting L-BFGS training")
        eng = eng if eng is not None else self._get_lbfgs_engine()
        flat = self._flat()
        bar = tqdm(total=newton_iter, disable=not (self.verbose and ctx.rank == 0), desc="L-BFGS")

        def on_eval(it, f):
            if self.metrics is not None and (it % self.log_every == 0 or it == newton_iter):
                self.metrics.log("lbfgs", it, f)
            if it % 10 == 0 or it == newton_iter:
                bar.n = min(it, newton_iter)
                bar.set_postfix(loss=f)
                bar.refresh()

        if newton_eager and self._use_device_lbfgs():
            from ..fit import _use_graphs
            from ..optimizers import lbfgs_device

            def on_poll(opt):
                ctx.check_health()   # a peer all-reduce timeout inside the L-BFGS graph
                polled = getattr(opt, "polled", None)   # the pipelined poll's host snapshot
                if polled is not None:
                    it, f = polled["n_iter"], polled["f"]
                else:
                    it = opt.n_iter
                    f = float(opt.st[lbfgs_device.F])
                if self.metrics is not None:
                    self.metrics.log("lbfgs", it, f)
                bar.n = min(it, newton_iter)
                bar.set_postfix(loss=f)
                bar.refresh()

            opt = lbfgs_device.minimize(eng.evaluate_fg, flat.data, newton_iter, lr=0.8,
                                        all_reduce=ctx.all_reduce_ if ctx.is_distributed else None,
                                        capture_all_reduce=ctx.capturable(flat.numel() + 1),
                                        use_graph=_use_graphs(self.device),
                                        poll_every=max(1, min(int(self.log_every), 64)), on_poll=on_poll,
                                        stop=stop, images=eng.image_target()
                                        if os.environ.get("TDQ_LBFGS_IMAGES", "1") != "0" else None)
            ctx.check_health()
            with torch.no_grad():
                flat.copy_(opt.best_x)
            self.min_loss["l-bfgs"] = opt.min_loss
            self.best_epoch["l-bfgs"] = opt.best_epoch
            self.lbfgs_state = opt
            info = {"impl": "device", "n_iter": opt.n_iter, "func_evals": opt.func_eval, "reason": opt.reason}
        elif newton_eager:
            from ..optimizers.lbfgs import Struct
            state = Struct()
            x, _, fe, best_w, min_loss, best_epoch = eager_lbfgs(
                eng, flat.detach().clone(), state=state, maxIter=newton_iter, learningRate=0.8, on_eval=on_eval,
                stop=stop)
            ctx.check_health()
            with torch.no_grad():
                flat.copy_(best_w)
            self.min_loss["l-bfgs"] = float(min_loss)
            self.best_epoch["l-bfgs"] = int(best_epoch)
            info = {"impl": "host", "n_iter": int(getattr(state, "nIter", 0)), "func_evals": int(fe),
                    "reason": getattr(state, "reason", "?")}
        else:
            # the reference's graph-mode L-BFGS (tfp lbfgs_minimize, fit.py:107-122): line-search
            # L-BFGS with 10 pairs and tolerance 1e-20, state on the device (optimizers/lbfgs_wolfe.py)
            from ..fit import _use_graphs
            from ..optimizers import lbfgs_wolfe
            prec = getattr(getattr(eng, "program", None), "precision", None)
            prec = prec if getattr(getattr(eng, "program", None), "backend", None) == "hip" else "fp32"
            opt = lbfgs_wolfe.minimize(eng.evaluate_fg, flat.data, newton_iter,
                                       all_reduce=ctx.all_reduce_ if ctx.is_distributed else None,
                                       capture_all_reduce=ctx.capturable(flat.numel() + 1),
                                       use_graph=_use_graphs(self.device), on_iter=on_eval,
                                       hz_eps=lbfgs_wolfe.hz_eps_for(prec))
            ctx.check_health()
            self.min_loss["l-bfgs"] = float(opt.min_loss)
            self.best_epoch["l-bfgs"] = int(opt.n_iter)
            info = {"impl": "strong-wolfe" + (" (device)" if opt.use_graph else ""), "n_iter": int(opt.n_iter),
                    "hz_eps": opt.hz_eps,
                    "func_evals": int(opt.func_eval), "reason": opt.reason, "restarts": int(opt.n_restarts)}
        bar.close()
        self._best_flat["l-bfgs"] = flat.detach().clone()
        self.best_model["l-bfgs"] = _FlatModel(self.u_model, self._best_flat["l-bfgs"])
        info["stop"] = stop
        return info

    def _select_overall(self, start_epoch, tf_iter):
        if self.min_loss["adam"] <= self.min_loss["l-bfgs"]:
            key, off = "adam", 0
        else:
            key, off = "l-bfgs", tf_iter
        self.min_loss["overall"] = self.min_loss[key]
        self.best_epoch["overall"] = self.best_epoch[key] + off if self.best_epoch[key] >= 0 else -1
        if key in self._best_flat:
            self._best_flat["overall"] = self._best_flat[key]
            self.best_model["overall"] = _FlatModel(self.u_model, self._best_flat[key])

    # ================================================================== outputs =========
    @property
    def losses(self):
        """Per-epoch loss history: list of dicts (term name -> value, plus 'Total Loss')."""
        st = self._state
        if st is None or st["hist"] is None:
            return []
        n = int(st["epoch_host"])
        h = st["hist"][:n].detach().cpu().numpy()
        names = [t.name for t in self.program().terms]
        out = []
        for row in h:
            d = {nm: float(v) for nm, v in zip(names, row[1:])}
            d["Total Loss"] = float(row[0])
            out.append(d)
        return out

    def predict(self, X_star, best_model=False, chunk=65536):
        params = None
        if best_model:
            if "overall" not in self._best_flat:
                raise ValueError("no best model recorded yet (call fit first)")
            params = self._best_flat["overall"]
        X = torch.as_tensor(np.asarray(X_star) if not torch.is_tensor(X_star) else X_star,
                            dtype=torch.float32).to(self.device)
        # u is the value stream of the same jet launch that computes the residual's derivatives
        # (HIP kernels on the hip backend), in bf16x3 when the solver trains in bf16 (the
        # L-BFGS phase's program, usually built already): prediction error ~1e-5, not bf16's ~1e-3
        prog = self.program(precision="bf16x3" if self.precision == "bf16" else None)
        vals = []
        f = prog.residual_on(self.f_model, X, params=params, chunk=chunk, values=vals)
        if vals and all(v is not None for v in vals):
            u = torch.cat(vals, dim=0)
        else:
            with torch.no_grad():
                u = torch.cat([self.u_model(X[i:i + chunk], params=params)
                               for i in range(0, X.shape[0], chunk)], dim=0)
        f_np = [x.cpu().numpy() for x in f]
        return u.cpu().numpy(), (f_np[0] if len(f_np) == 1 else tuple(f_np))

    def save(self, path, include_state=True):
        checkpoint.save_solver(self, path, include_state=include_state)

    def load_model(self, path, compile_model=False, restore_state=False):
        checkpoint.load_into_solver(self, path, restore_state=restore_state)

    def resume(self, path):
        """Load weights AND training state (SA weights, Adam moments, epoch, best snapshot)."""
        checkpoint.load_into_solver(self, path, restore_state=True)
