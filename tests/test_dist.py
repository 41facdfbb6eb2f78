"""Data parallelism without a cluster: gloo on CPU, world_size 2 and 4.

Asserts that sharded DP (collocation points + SA weights split by rank, replicated BC terms
scaled by 1/world, one flat all-reduce) reproduces the single-process full-batch loss,
gradients and Adam trajectory, and that L-BFGS runs under DP.
"""
import os

import pytest
import torch
import torch.multiprocessing as mp

import tensordiffeq_amd as tdq


def _free_port():
    from tensordiffeq_amd.parallel.dist import free_port
    return free_port()


def _build(dist):
    from tests.test_solver import allen_cahn
    D, bcs, f, kw = allen_cahn(n_f=301)
    torch.manual_seed(0)
    m = tdq.CollocationSolverND(verbose=False)
    m.compile([2, 12, 12, 1], f, D, bcs, backend="jet", device="cpu", dist=dist, **kw)
    return m


def _np(t):
    """Queue payloads travel as numpy: a torch tensor would be sent as a shared-memory handle that
    disappears once the sending process exits (FileNotFoundError in the receiver)."""
    return t.detach().cpu().numpy().copy()


def _t(a):
    return torch.from_numpy(a)


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    from tensordiffeq_amd.parallel import dist as pdist
    pdist.reset_context()
    ctx = pdist.init_distributed(backend="gloo", device="cpu")
    m = _build(True)
    eng = m._get_engine(None, 10)
    loss, grads, terms = eng._phase_a()
    loss, grads, terms = eng._reduce(loss, grads, terms)
    res = {"loss": float(loss), "gflat": _np(grads[0]), "glam_bc": _np(grads[2])}
    m.fit(tf_iter=5)
    res["flat_after"] = _np(m.u_model.flat)
    res["hist"] = [h["Total Loss"] for h in m.losses]
    m.fit(newton_iter=3)
    res["flat_lbfgs"] = _np(m.u_model.flat)
    m.fit(newton_iter=4, newton_eager=False)      # line-search L-BFGS through the same all-reduce
    res["flat_wolfe"] = _np(m.u_model.flat)
    res["wolfe_evals"] = m.fit_info["lbfgs"]["func_evals"]
    if rank == 0:
        q.put(res)
    ctx.barrier()
    pdist.destroy()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 4])
def test_dp_gloo_matches_single_process(world):
    ref = _build(False)
    eng = ref._get_engine(None, 10)
    loss, grads, terms = eng._phase_a()
    ref.fit(tf_iter=5)
    ref_hist = [h["Total Loss"] for h in ref.losses]
    ref_flat = ref.u_model.flat.detach().clone()
    ref.fit(newton_iter=3)
    ref_lbfgs = ref.u_model.flat.detach().clone()
    ref.fit(newton_iter=4, newton_eager=False)
    ref_wolfe = ref.u_model.flat.detach().clone()

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=280)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res["loss"] == pytest.approx(float(loss), rel=1e-5)
    assert torch.allclose(_t(res["gflat"]), grads[0], rtol=1e-4, atol=1e-6)
    assert torch.allclose(_t(res["glam_bc"]), grads[2], rtol=1e-4, atol=1e-7)
    assert res["hist"] == pytest.approx(ref_hist, rel=1e-4)
    assert torch.allclose(_t(res["flat_after"]), ref_flat, atol=1e-5)
    assert torch.allclose(_t(res["flat_lbfgs"]), ref_lbfgs, atol=1e-4)
    assert torch.allclose(_t(res["flat_wolfe"]), ref_wolfe, atol=1e-4)
    assert res["wolfe_evals"] == ref.fit_info["lbfgs"]["func_evals"]


def _worker_batched(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    from tensordiffeq_amd.parallel import dist as pdist
    pdist.reset_context()
    ctx = pdist.init_distributed(backend="gloo", device="cpu")
    m = _build(True)          # N_f = 301 over 2 ranks: shards of 151 and 150 points
    batches = m.minibatches(50)
    m.fit(tf_iter=2, batch_sz=50)
    q.put({"rank": rank, "n_local": m.X_f_local.shape[0], "batches": batches,
           "epochs": int(m._state["epoch_host"]), "flat": _np(m.u_model.flat),
           "lam": _np(m.lambdas[0])})
    ctx.barrier()
    pdist.destroy()


@pytest.mark.timeout(300)
def test_dp_minibatch_uneven_shards():
    """Uneven shards + batch_sz: every rank runs the same number of minibatch steps (one
    all-reduce each), so the run completes and theta stays identical across ranks."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_batched, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=280) for _ in range(2)], key=lambda r: r["rank"])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r["n_local"] for r in res] == [151, 150]
    assert res[0]["batches"] == res[1]["batches"] == [(0, 50), (50, 100), (100, 150)]
    assert res[0]["epochs"] == res[1]["epochs"] == 6
    assert (res[0]["flat"] == res[1]["flat"]).all()
    assert res[0]["lam"].shape == (151, 1) and res[1]["lam"].shape == (150, 1)


def test_minibatches_single_process():
    m = _build(False)
    assert m.minibatches(None) == [None]
    assert m.minibatches(301) == [None]
    assert m.minibatches(100) == [(0, 100), (100, 200), (200, 300)]
    with pytest.raises(ValueError):
        m.minibatches(0)


def _discovery_problem():
    import math
    import numpy as np
    x = np.linspace(-1, 1, 21)
    t = np.linspace(0, 1, 9)
    X, T = np.meshgrid(x, t)
    xs, ts = X.reshape(-1, 1), T.reshape(-1, 1)            # 189 points: uneven shards
    u = np.sin(math.pi * xs) * np.exp(-0.5 * ts)

    def f_model(u_model, var, x, t):
        uu = u_model(torch.cat([x, t], 1))
        return tdq.grad(uu, t) - var[0] * tdq.grad(tdq.grad(uu, x), x)

    return f_model, xs, ts, u


def _build_discovery(dist):
    import numpy as np
    f_model, xs, ts, u = _discovery_problem()
    torch.manual_seed(0)
    var = [tdq.Variable(0.1)]
    cw = np.linspace(0.5, 1.5, xs.shape[0]).reshape(-1, 1).astype(np.float32)
    m = tdq.DiscoveryModel(verbose=False)
    m.compile([2, 10, 10, 1], f_model, [xs, ts], u, var, col_weights=cw, backend="jet", device="cpu",
              dist=dist)
    return m, var


def _worker_discovery(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    from tensordiffeq_amd.parallel import dist as pdist
    pdist.reset_context()
    ctx = pdist.init_distributed(backend="gloo", device="cpu")
    m, var = _build_discovery(True)
    m.fit(tf_iter=4)
    res = {"rank": rank, "flat": _np(m.u_model.flat), "var": float(var[0].detach()),
           "cw": _np(m.col_weights), "lo": m._lo, "hi": m._hi}
    q.put(res)
    ctx.barrier()
    pdist.destroy()


@pytest.mark.timeout(300)
def test_discovery_dp_gloo_matches_single_process():
    """DiscoveryModel under DP: data points and their SA collocation weights sharded, network and
    PDE coefficients all-reduced - same trajectory as the single-process full batch."""
    ref, rvar = _build_discovery(False)
    ref.fit(tf_iter=4)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_discovery, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=280) for _ in range(2)], key=lambda r: r["rank"])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert (res[0]["flat"] == res[1]["flat"]).all()
    assert torch.allclose(_t(res[0]["flat"]), ref.u_model.flat.detach(), atol=1e-5)
    assert res[0]["var"] == pytest.approx(float(rvar[0].detach()), rel=1e-4, abs=1e-7)
    cw = torch.cat([_t(r["cw"]) for r in res])
    assert torch.allclose(cw, ref.col_weights.detach(), atol=1e-5)


def _forced_worker(q):
    os.environ.update(TDQ_FORCE_DP="1", WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", TDQ_LBFGS="device")
    os.environ.pop("MASTER_PORT", None)
    torch.set_num_threads(1)
    from tensordiffeq_amd.parallel import dist as pdist
    pdist.reset_context()
    ctx = pdist.init_distributed(backend="gloo", device="cpu")
    assert ctx.is_distributed and ctx.forced and ctx.world == 1 and not ctx.graph_collectives
    m = _build(True)
    m.fit(tf_iter=5, newton_iter=4)
    # plain numbers / numpy: a torch tensor would travel as a shared-memory handle that is gone
    # once this process exits
    q.put({"hist": [h["Total Loss"] for h in m.losses], "flat": m.u_model.flat.detach().numpy().copy(),
           "lbfgs": m.min_loss["l-bfgs"], "red": len(m._get_engine(None, 1).red_idx)})
    pdist.destroy()


@pytest.mark.timeout(300)
def test_forced_dp_world1_matches_single_process(monkeypatch):
    """TDQ_FORCE_DP=1: a real process group at world 1 runs the DP step (bucket all-reduce, SA
    residual weights treated as sharded) and reproduces the single-process trajectory."""
    monkeypatch.setenv("TDQ_LBFGS", "device")
    ref = _build(False)
    ref.fit(tf_iter=5, newton_iter=4)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_forced_worker, args=(q,))
    p.start()
    res = q.get(timeout=280)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert res["hist"] == pytest.approx([h["Total Loss"] for h in ref.losses], rel=1e-6)
    assert torch.allclose(torch.from_numpy(res["flat"]), ref.u_model.flat.detach(), rtol=1e-6, atol=1e-7)
    assert res["lbfgs"] == pytest.approx(ref.min_loss["l-bfgs"], rel=1e-6)
    assert res["red"] == 2   # theta + the IC's SA weights; residual SA weights stay local


def _g_square(lam):
    return lam * lam


def _build_type2(dist, with_g=False):
    from tests.test_solver import allen_cahn
    D, bcs, f, _ = allen_cahn(n_f=301, sa=False)
    g = torch.Generator().manual_seed(3)
    kw = dict(Adaptive_type=2, dict_adaptive={"residual": [True], "BCs": [False, False]},
              init_weights={"residual": [torch.rand(301, 1, generator=g)], "BCs": [None, None]})
    if with_g:   # g_MSE: element-wise g(lam) f^2 - the weights shard with their points
        kw["g"] = _g_square
    torch.manual_seed(0)
    m = tdq.CollocationSolverND(verbose=False)
    m.compile([2, 12, 12, 1], f, D, bcs, backend="jet", device="cpu", dist=dist, **kw)
    return m


def _worker_type2(rank, world, port, q, with_g=False):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    from tensordiffeq_amd.parallel import dist as pdist
    pdist.reset_context()
    ctx = pdist.init_distributed(backend="gloo", device="cpu")
    m = _build_type2(True, with_g)
    m.fit(tf_iter=5)
    lam = m.lambdas[0].detach()
    if with_g:   # sharded: gather the ranks' slices in rank order
        import torch.distributed as tdist
        sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        tdist.all_gather(sizes, torch.tensor([lam.shape[0]]))
        mx = int(max(sizes))
        buf = [torch.zeros(mx, 1) for _ in range(world)]
        pad = torch.zeros(mx, 1)
        pad[:lam.shape[0]] = lam
        tdist.all_gather(buf, pad)
        lam = torch.cat([b[:int(n)] for b, n in zip(buf, sizes)])
    res = {"hist": [h["Total Loss"] for h in m.losses], "flat": _np(m.u_model.flat), "lam": _np(lam),
           "lam_local": int(m.lambdas[0].shape[0])}
    if rank == 0:
        q.put(res)
    ctx.barrier()
    pdist.destroy()


@pytest.mark.timeout(300)
def test_dp_adaptive_type2_per_point_weights():
    """Adaptive_type 2 ("loss-weights": (sum_i w_i) * mean(r^2), reference utils.py:38-44) with
    per-point residual weights under DP: the weights stay replicated (their sum multiplies every
    rank's partial mean) and their gradient is all-reduced - the trajectory equals single-process."""
    ref = _build_type2(False)
    ref.fit(tf_iter=5)
    ref_hist = [h["Total Loss"] for h in ref.losses]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_type2, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=280)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res["hist"] == pytest.approx(ref_hist, rel=1e-4)
    assert torch.allclose(_t(res["flat"]), ref.u_model.flat.detach(), atol=1e-5)
    assert torch.allclose(_t(res["lam"]), ref.lambdas[0].detach(), atol=1e-5)


@pytest.mark.timeout(300)
def test_dp_adaptive_type2_with_g_shards_weights():
    """Adaptive_type 2 with ``g`` uses g_MSE (element-wise g(lam) f^2), so the per-point
    weights are sharded with their points (replicated ones failed to broadcast against the rank's
    residual); the trajectory and the gathered weights equal single-process training."""
    ref = _build_type2(False, with_g=True)
    ref.fit(tf_iter=5)
    ref_hist = [h["Total Loss"] for h in ref.losses]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_type2, args=(r, 2, port, q, True)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=280)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res["lam_local"] < 301
    assert res["hist"] == pytest.approx(ref_hist, rel=1e-4)
    assert torch.allclose(_t(res["flat"]), ref.u_model.flat.detach(), atol=1e-5)
    assert torch.allclose(_t(res["lam"]), ref.lambdas[0].detach(), atol=1e-5)
