"""Device-resident L-BFGS (optimizers/lbfgs_device.py, csrc/lbfgs.hip).

CPU: the torch mirror of the update kernels against the host port ``eager_lbfgs`` (itself the
lua-port semantics of reference optimizers.py:107-308) on a quadratic, Rosenbrock, the stopping
tests, the solver integration and DP over gloo.  GPU: the native kernels against the mirror step
by step (history-ring wrap-around included), graph replay against eager launches (bitwise), and
the solver on the HIP path against the host-driven optimizer.
"""
import math
import os

import pytest
import torch
import torch.multiprocessing as mp

from tensordiffeq_amd.optimizers import eager_lbfgs
from tensordiffeq_amd.optimizers import lbfgs_device as LD


def _quadratic(p=40, q=60, seed=0, device="cpu"):
    g = torch.Generator().manual_seed(seed)
    M = (torch.randn(q, p, generator=g) / math.sqrt(q)).to(device)
    b = torch.randn(q, generator=g).to(device)

    def fg(x):
        r = M @ x - b
        return 0.5 * (r @ r), M.T @ r
    xs = torch.linalg.lstsq(M.double().cpu(), b.double().cpu().unsqueeze(1)).solution.squeeze(1)
    r = M.double().cpu() @ xs - b.double().cpu()
    fg.f_opt = float(0.5 * (r @ r))
    return fg


def _evaluator(fg_fn, x):
    def evaluate():
        f, g = fg_fn(x)
        return torch.cat([g.reshape(-1), f.reshape(1)]).float().contiguous()
    return evaluate


def test_mirror_matches_eager_lbfgs_on_quadratic():
    fg = _quadratic()
    x0 = torch.zeros(40)
    _, f_hist, _, _, fmin, _ = eager_lbfgs(fg, x0.clone(), maxIter=25, learningRate=0.8)
    x = x0.clone()
    opt = LD.minimize(_evaluator(fg, x), x, 25, lr=0.8, use_graph=False)
    hist = opt.history()
    ref = [float(v) for v in f_hist]
    # the host port skips the evaluation after its last step: compare the evaluated prefix
    assert len(hist) == 26
    assert hist[:25] == pytest.approx(ref[:25], rel=1e-3, abs=1e-6)
    assert opt.reason == LD.REASONS[3] and opt.n_iter == 25 and opt.func_eval == 26
    assert opt.min_loss <= fmin * (1 + 1e-3)
    assert float(fg(opt.best_x)[0]) == pytest.approx(opt.min_loss, rel=1e-4)
    assert hist[-1] - fg.f_opt < 0.2 * (hist[0] - fg.f_opt)


def test_mirror_history_ring_wraps():
    fg = _quadratic(p=30, q=45, seed=3)
    x = torch.zeros(30)
    opt = LD.minimize(_evaluator(fg, x), x, 40, m=4, use_graph=False)
    assert int(opt.st[LD.K]) == 4
    h = opt.history()
    assert min(h) - fg.f_opt < 0.05 * (h[0] - fg.f_opt)


def test_mirror_rosenbrock():
    def fg(x):
        a, b = x[0].double(), x[1].double()
        f = (1 - a) ** 2 + 100 * (b - a * a) ** 2
        g = torch.stack([-2 * (1 - a) - 400 * a * (b - a * a), 200 * (b - a * a)])
        return f.float(), g.float()
    x = torch.tensor([-1.2, 1.0])
    f0 = float(fg(x)[0])
    opt = LD.minimize(_evaluator(fg, x), x, 400, use_graph=False)
    assert opt.min_loss < 1e-3 * f0


def test_stopping_tests():
    # optimal start: tolFun on the initial gradient, no step taken
    x = torch.zeros(3)
    opt = LD.minimize(lambda: torch.zeros(4), x, 10, use_graph=False)
    assert opt.reason == LD.REASONS[1] and opt.n_iter == 0 and torch.equal(x, torch.zeros(3))
    # NaN loss after two evaluations
    calls = [0]

    def nan_eval():
        calls[0] += 1
        v = torch.ones(4)
        v[-1] = float("nan") if calls[0] > 2 else 10.0 - calls[0]
        return v
    x = torch.zeros(3)
    opt = LD.minimize(nan_eval, x, 10, use_graph=False)
    assert opt.reason == LD.REASONS[2] and opt.n_iter == 2 and opt.min_loss == 8.0
    # the best iterate is the one that produced the lowest loss (x after the first step)
    assert torch.allclose(opt.best_x, torch.full((3,), -1.0 / 3.0))


def _offset_quadratic():
    base = _quadratic(p=20, q=30, seed=5)

    def fg(x):
        f, g = base(x)
        return f + 5.0, g   # minimum 5 + f_opt: never |f| < tolX
    return fg


@pytest.mark.parametrize("stop", ["fixed", "legacy"])
def test_stop_modes(stop):
    """``stop="fixed"``: |f - f_old| < tolX ends a stagnated run; ``"legacy"``: the reference's
    effective |f| < tolX (optimizers.py:273) never fires on a loss bounded away from 0, so the
    run only ends on maxIter or another test.  Host port and device mirror agree on the reason."""
    fg = _offset_quadratic()
    x = torch.zeros(20)
    opt = LD.minimize(_evaluator(fg, x), x, 400, use_graph=False, stop=stop)
    from tensordiffeq_amd.optimizers.lbfgs import Struct
    st = Struct()
    eager_lbfgs(fg, torch.zeros(20), state=st, maxIter=400, learningRate=0.8, stop=stop)
    if stop == "fixed":
        assert opt.reason == LD.REASONS[4] and opt.n_iter < 400
    else:
        assert opt.reason != LD.REASONS[4]
    assert st.reason == opt.reason


def test_stop_mode_legacy_runs_longer():
    fg = _offset_quadratic()
    n = {}
    for stop in ("fixed", "legacy"):
        x = torch.zeros(20)
        n[stop] = LD.minimize(_evaluator(fg, x), x, 400, use_graph=False, stop=stop).n_iter
    assert n["legacy"] >= n["fixed"]


def test_solver_records_lbfgs_stop(monkeypatch):
    from tests.test_solver import compiled
    m = compiled("jet", problem="ac", lbfgs_stop="legacy")
    m.fit(tf_iter=2, newton_iter=4)
    info = m.fit_info["lbfgs"]
    assert info["stop"] == "legacy" and info["n_iter"] == 4 and info["reason"] == LD.REASONS[3]
    assert info["wall_s"] > 0


def test_solver_device_lbfgs_matches_host(monkeypatch):
    from tests.test_solver import compiled
    res = {}
    for impl in ("host", "device"):
        monkeypatch.setenv("TDQ_LBFGS", impl)
        m = compiled("jet", problem="ac")
        m.fit(tf_iter=5, newton_iter=15)
        res[impl] = m.min_loss["l-bfgs"]
        assert math.isfinite(res[impl])
        if impl == "device":
            assert m.lbfgs_state.n_iter == 15
            f_best = float(m.update_loss().detach())
            assert f_best == pytest.approx(m.min_loss["l-bfgs"], rel=1e-4)
    # identical algorithm; the device run also evaluates the last iterate
    assert res["device"] <= res["host"] * (1 + 1e-3)
    assert res["device"] >= 0.5 * res["host"]


def _free_port():
    from tensordiffeq_amd.parallel.dist import free_port
    return free_port()


def _dp_worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), TDQ_LBFGS="device")
    torch.set_num_threads(1)
    from tensordiffeq_amd.parallel import dist as pdist
    from tests.test_dist import _build
    pdist.reset_context()
    ctx = pdist.init_distributed(backend="gloo", device="cpu")
    m = _build(True)
    m.fit(tf_iter=3, newton_iter=6)
    out = {"flat": m.u_model.flat.detach().clone(), "loss": m.min_loss["l-bfgs"]}
    if rank == 0:
        q.put(out)
    ctx.barrier()
    pdist.destroy()


@pytest.mark.timeout(300)
def test_device_lbfgs_under_dp_matches_single_process(monkeypatch):
    from tests.test_dist import _build
    monkeypatch.setenv("TDQ_LBFGS", "device")
    ref = _build(False)
    ref.fit(tf_iter=3, newton_iter=6)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=280)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res["loss"] == pytest.approx(ref.min_loss["l-bfgs"], rel=1e-4)
    assert torch.allclose(res["flat"], ref.u_model.flat.detach(), atol=1e-4)


# ------------------------------------------------------------------ GPU ---------------------
@pytest.mark.gpu
@pytest.mark.parametrize("m", [5, 50])
def test_native_kernels_match_mirror(m):
    from tensordiffeq_amd.ops import _lib
    _lib.load(required=True)
    fg = _quadratic(p=3000, q=4000, seed=1, device="cuda")
    x_n = torch.zeros(3000, device="cuda")
    x_m = x_n.clone()
    on = LD.DeviceLBFGS(x_n, m=m, max_iter=40)
    om = LD.DeviceLBFGS(x_m, m=m, max_iter=40)
    assert on.native
    om.native = False
    ev_n, ev_m = _evaluator(fg, x_n), _evaluator(fg, x_m)
    on.update(ev_n())
    om.update(ev_m())
    while om.active():
        on.axpy()
        on.update(ev_n())
        om.axpy()
        om.update(ev_m())
    torch.cuda.synchronize()
    assert not on.active()
    assert on.n_iter == om.n_iter and on.reason == om.reason
    for k in (LD.K, LD.HEAD, LD.FEVAL, LD.BESTEP):
        assert float(on.st[k]) == float(om.st[k])
    assert torch.allclose(on.fhist, om.fhist, rtol=1e-4, atol=1e-6, equal_nan=True)
    assert ((x_n - x_m).norm() / x_m.norm()).item() < 1e-4
    assert ((on.best_x - om.best_x).norm() / om.best_x.norm()).item() < 1e-4


@pytest.mark.gpu
def test_graph_replay_matches_eager_launches():
    fg = _quadratic(p=2000, q=2500, seed=2, device="cuda")
    outs = []
    for use_graph in (False, True):
        x = torch.zeros(2000, device="cuda")
        opt = LD.minimize(_evaluator(fg, x), x, 60, m=10, use_graph=use_graph, poll_every=7)
        torch.cuda.synchronize()
        outs.append((x.clone(), opt.history(), opt.n_iter, opt.best_x.clone()))
    assert outs[0][2] == outs[1][2] == 60
    assert torch.equal(outs[0][0], outs[1][0])
    assert outs[0][1] == outs[1][1]
    assert torch.equal(outs[0][3], outs[1][3])


@pytest.mark.gpu
def test_solver_device_lbfgs_on_hip_path(monkeypatch):
    import bench
    res = {}
    for impl in ("host", "device"):
        monkeypatch.setenv("TDQ_LBFGS", impl)
        m = bench.build_problem(2048, 1, "hip", torch.device("cuda", 0), False)
        assert m.active_backend == "hip"
        m.fit(tf_iter=20)
        m.fit(newton_iter=30)
        res[impl] = m.min_loss["l-bfgs"]
    assert res["device"] == pytest.approx(res["host"], rel=5e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("use_graph,p", [(False, 3000), (True, 3000), (True, 60000)])
def test_fused_update_matches_five_launch_path(use_graph, p, monkeypatch):
    """The two-launch update (dots + logic, direction + descent test + step, each finished by the
    block arriving last on its counter tree) reproduces the five-launch path bit for bit: iterate,
    loss history, best iterate, stop reason - incl. the history-ring wrap-around.  p = 60000:
    195 dots blocks and 938 direction blocks, every group of the 32-way tree several deep."""
    fg = _quadratic(p=p, q=4000 if p <= 3000 else 300, seed=4, device="cuda")
    outs = []
    for fused in ("1", "0"):
        monkeypatch.setenv("TDQ_LBFGS_FUSED", fused)
        x = torch.zeros(p, device="cuda")
        opt = LD.minimize(_evaluator(fg, x), x, 80, m=12, use_graph=use_graph, poll_every=9)
        torch.cuda.synchronize()
        assert opt.fused == (fused == "1")
        outs.append((x.clone(), opt.history(), opt.n_iter, opt.best_x.clone(), opt.reason, opt.st.clone()))
    a, b = outs
    assert a[2] == b[2] and a[4] == b[4]
    assert torch.equal(a[0], b[0]) and torch.equal(a[3], b[3])
    assert a[1] == b[1]
    assert torch.equal(a[5], b[5])


@pytest.mark.gpu
def test_fused_update_descent_stop_restores_x(monkeypatch):
    """A gradient the direction cannot descend along (g.d > -tolX from the first step): the fused
    path stops with the same reason and leaves x where the five-launch path does (the speculative
    step is undone)."""
    outs = []
    for fused in ("1", "0"):
        monkeypatch.setenv("TDQ_LBFGS_FUSED", fused)
        x = torch.ones(5000, device="cuda")
        # tiny gradient: |g|_1 > tolFun but g.d = -|g|^2 > -tolX
        evaluate = lambda: torch.cat([torch.full((5000,), 1e-9, device="cuda"),
                                      torch.ones(1, device="cuda")]).contiguous()
        opt = LD.minimize(evaluate, x, 10, use_graph=False)
        torch.cuda.synchronize()
        outs.append((x.clone(), opt.reason, opt.n_iter))
    assert outs[0][1] == outs[1][1] == LD.REASONS[5]
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][0], torch.ones(5000, device="cuda"))


@pytest.mark.gpu
def test_device_lbfgs_images_from_update_match_pack(monkeypatch):
    """The fused update scatters the next x into the one-launch objective's weight images
    (TDQ_LBFGS_IMAGES, default on) instead of a pack launch per evaluation: the same trajectory,
    bit for bit (AC-SA, bf16x3 objective)."""
    import bench
    from tensordiffeq_amd.ops import fused_step
    hist = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("TDQ_LBFGS_IMAGES", flag)
        m = bench.build_problem(4096, 1, "hip", torch.device("cuda", 0), False, "bf16", newton_precision="bf16x3")
        m.fit(tf_iter=200)
        m.fit(newton_iter=60)
        assert fused_step.for_program(m.program(precision="bf16x3")) is not None
        hist[flag] = (m.lbfgs_state.history(), m.u_model.flat.detach().clone())
    assert hist["1"][0] == hist["0"][0]
    assert torch.equal(hist["1"][1], hist["0"][1])
