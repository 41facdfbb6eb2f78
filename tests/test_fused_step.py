"""One-launch residual training step (ops/fused_step.py, csrc/jet_fused.h MODE 2).

CPU: the generated kernels (headers + the program's loss as ``GenLoss``; the bf16 step and the
bf16x3 objective) compile with hipRTC for gfx950 for several traced programs, and eligibility is
decided from the program's layout.
GPU: the fused step's loss, SA-weight gradients and parameter gradient match the separate-launch
step (saved-activation kernels + specialized loss kernel) at the bf16 level, and a short training
run follows the same trajectory.
"""
import ctypes

import pytest
import torch

import tensordiffeq_amd as tdq
from tensordiffeq_amd import fusion
from tests.test_loss_jit import _model
from tests.test_solver import allen_cahn, burgers


def _deep(problem, layers):
    torch.manual_seed(0)
    m = tdq.CollocationSolverND(verbose=False)
    if problem == "burgers":
        D, bcs, f = burgers(n_f=400)
        m.compile(layers, f, D, bcs, backend="jet", device="cpu")
    else:
        D, bcs, f, kw = allen_cahn(n_f=400)
        if problem == "ac_g":
            kw["g"] = lambda lam: lam ** 2 + 0.5 * torch.exp(-lam)
        m.compile(layers, f, D, bcs, backend="jet", device="cpu", **kw)
    return m


def _compile_ok(src):
    from tensordiffeq_amd.ops import _lib, fused_step
    lib = _lib.load()
    code, size = ctypes.c_void_p(0), ctypes.c_longlong(0)
    log = ctypes.create_string_buffer(16384)
    rc = lib.tdq_rtc_compile_ex(src.encode(), b"t.hip", b"gfx950", fused_step.RTC_OPTS.encode(), ctypes.byref(code),
                                ctypes.byref(size), log, len(log))
    assert rc == 0, log.value.decode()[:3000]
    assert size.value > 0
    lib.tdq_rtc_free(code)


@pytest.mark.parametrize("problem,layers", [("ac", [2, 128, 128, 128, 128, 1]), ("ac_g", [2, 128, 128, 128, 1]),
                                            ("burgers", [2, 128, 128, 128, 128, 1]), ("ac", [2, 128, 128, 1])])
def test_fused_step_source_compiles(problem, layers):
    from tensordiffeq_amd.ops import _lib, fused_step, jet_hip
    from tensordiffeq_amd.ops.jet_mlp import hip_config
    from tensordiffeq_amd.ops.loss_fused import FusedLossOp
    if not _lib.available():
        pytest.skip("native library not built")
    m = _deep(problem, layers)
    prog = m.program()
    fl = fusion.build(prog, m.lambdas)
    op = FusedLossOp(fl, prog, m.lambdas, fusion.scalar_values(fl, m.lambdas, None), fl.lam_offsets)
    # the residual group is the last group, alone on the last segment
    last = len(prog.segments) - 1
    assert fl.groups[-1].segs == [last]
    cfg = hip_config(prog.net, prog.plan, "bf16")
    lib = _lib.load()
    lds = lib.tdq_jet_fused_lds(cfg["d_in"], jet_hip._warg(cfg), cfg["d_out"], cfg["n_hidden"], cfg["S"], 0)
    if lds < 0:   # a 1-MFMA-layer net ([2, 128, 128, 1]): MODE 2 needs two
        assert cfg["n_hidden"] - 1 < 2
        return
    spec = jet_hip.stream_spec(prog.plan)
    nso = sum(1 for s in range(cfg["S"]) if spec[3 * s] == 2)
    layout, pos = [], 0
    for gr in fl.groups:
        ns = len(gr.segs)
        pos += pos % 2 if ns == 2 else 0
        layout.append((gr.program, pos, ns, gr.n))
        pos += ns * gr.n
    gen = fused_step.gen_loss(layout, op.n_terms, op.n_terms + op.n_scal, cfg["S"], spec=spec, d_in=cfg["d_in"])
    assert "JV(" in gen and "UB(" in gen
    if problem == "ac":   # the periodic pair group reads its partner point
        assert "t + 1" in gen
    _compile_ok(fused_step.kernel_source(cfg["S"], nso, cfg["n_hidden"] - 1, lds, gen))
    lds3 = lib.tdq_jet_fused_lds(cfg["d_in"], jet_hip._warg(cfg), cfg["d_out"], cfg["n_hidden"], cfg["S"], 1)
    assert 0 < lds3 <= 160 * 1024, lds3
    _compile_ok(fused_step.kernel_source(cfg["S"], nso, cfg["n_hidden"] - 1, lds3, gen, lo=True))


def test_fused_step_not_on_cpu():
    from tensordiffeq_amd.ops import fused_step
    m = _model("ac", "cpu", "jet")
    prog = m.program()
    assert fused_step.ineligible(prog, getattr(prog, "fused_op", None)) is not None


# --------------------------------------------------------------------------- GPU ---------
def _acsa(n_f, seed=0, problem="ac-sa", precision="bf16"):
    import bench
    torch.manual_seed(seed)
    return bench.PROBLEMS[problem]["build"](n_f, 1, "hip", torch.device("cuda", 0), False, precision,
                                            layers=(2, 128, 128, 128, 128, 1))


@pytest.mark.gpu
@pytest.mark.parametrize("problem,n_f,mixed,precision", [("ac-sa", 50000, "split", "bf16"),
                                                         ("ac-sa", 3001, "split", "bf16"),
                                                         ("ac-baseline", 20000, "split", "bf16"),
                                                         ("ac-baseline", 20000, "1", "bf16"),
                                                         ("ac-sa", 50000, "split", "bf16x3"),
                                                         ("ac-sa", 3001, "split", "bf16x3")])
def test_fused_step_matches_separate_launches(problem, n_f, mixed, precision, monkeypatch):
    """One evaluation: every loss term, the theta gradient and the SA-weight gradients of the fused
    step vs the separate launches (saved-activation kernels + specialized loss kernel).  AC-SA runs
    every group in the fused launch (IC with SA weights, the periodic pairs, the residual);
    AC-baseline (order-4 periodic streams): split layout - every main-plan output fused, the
    u_xxx / u_xxxx outputs on the jet_hi side chain; layout "1" - the residual only."""
    monkeypatch.setenv("TDQ_FUSED_STEP_MIXED", mixed)
    from tensordiffeq_amd.fit import LossGradEngine
    from tensordiffeq_amd.ops import fused_step
    out = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("TDQ_FUSED_STEP", flag)
        m = _acsa(n_f, problem=problem, precision=precision)
        prog = m.program()
        fop = prog.fused_op
        fs = fused_step.for_program(prog)
        if flag == "1":
            assert fs is not None, prog.fused_step_reason
            assert fs.mixed == (problem == "ac-baseline")
            if fs.mixed:
                assert fs.layout == ("split" if mixed == "split" else "residual")
            assert fs.lo == (precision == "bf16x3")
        else:
            assert fs is None
        eng = LossGradEngine(m, prog, m.lambdas)
        fg = eng.evaluate_fg()
        torch.cuda.synchronize()
        out[flag] = (fg.double().cpu(), [d.double().cpu().clone() for d in fop.dlam], fop.losses.double().cpu().clone())
    g1, g0 = out["1"][0][:-1], out["0"][0][:-1]
    rel = ((g1 - g0).norm() / g0.norm()).item()
    terms = [(a.item(), b.item()) for a, b in zip(out["1"][2], out["0"][2])]
    print(f"FUSED_STEP {problem} n_f={n_f} {precision} terms {[(f'{a:.5e}', f'{b:.5e}') for a, b in terms]} grad rel {rel:.3e}")
    # bf16: the two kernel designs round different operands (layer 0's tanh form, slab precision);
    # bf16x3: both at the split-bf16 level
    tl, tg = (2e-2, 3e-2) if precision == "bf16" else (5e-5, 1e-4)
    for a, b in terms:
        assert abs(a - b) <= tl * abs(b) + 1e-6, terms
    assert rel < tg, rel
    for a, b in zip(out["1"][1], out["0"][1]):
        assert ((a - b).norm() / b.norm().clamp_min(1e-30)).item() < tg


@pytest.mark.gpu
def test_fused_step_training_trajectory(monkeypatch):
    """AC-SA 20k: 200 Adam steps (graphs + fused tail) with and without the fused step end at the
    same loss within the bf16 level."""
    hist = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("TDQ_FUSED_STEP", flag)
        m = _acsa(20000)
        m.fit(tf_iter=200)
        assert (getattr(m.program(), "_fused_step", None) is not None) == (flag == "1")
        hist[flag] = [h["Total Loss"] for h in m.losses]
    a, b = hist["1"], hist["0"]
    print(f"FUSED_STEP_TRAJ first {a[0]:.5e} / {b[0]:.5e} last {a[-1]:.5e} / {b[-1]:.5e}")
    assert abs(a[0] - b[0]) <= 2e-2 * abs(b[0])
    assert abs(a[-1] - b[-1]) <= 0.1 * abs(b[-1])


@pytest.mark.gpu
def test_fused_step_deterministic(monkeypatch):
    monkeypatch.setenv("TDQ_FUSED_STEP", "1")
    m = _acsa(20000)
    from tensordiffeq_amd.fit import LossGradEngine
    eng = LossGradEngine(m, m.program(), m.lambdas)
    a = eng.evaluate_fg().clone()
    b = eng.evaluate_fg().clone()
    assert torch.equal(a, b)
