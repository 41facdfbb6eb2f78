"""SolverConfig env overrides and JSONL metrics (CPU)."""
import math

import numpy as np
import pytest
import torch

import tensordiffeq_amd as tdq
from tensordiffeq_amd.config import SolverConfig
from tensordiffeq_amd.metrics import read_jsonl


def test_config_env_and_overrides(monkeypatch):
    monkeypatch.setenv("TDQ_PRECISION", "fp32")
    monkeypatch.setenv("TDQ_LOG_EVERY", "7")
    monkeypatch.setenv("TDQ_NO_GRAPH", "1")
    c = SolverConfig.from_env()
    assert c.precision == "fp32" and c.log_every == 7 and not c.graphs
    c = SolverConfig.from_env(precision="bf16x3", log_every=None)
    assert c.precision == "bf16x3" and c.log_every == 7
    with pytest.raises(ValueError):
        SolverConfig.from_env(backend="cuda")


def test_newton_precision_builds_separate_program(monkeypatch):
    """Per-phase jet precision: the L-BFGS engine gets its own program (and kernel family)."""
    from tensordiffeq_amd.boundaries import DomainND, dirichletBC
    monkeypatch.setenv("TDQ_NEWTON_PRECISION", "bf16x3")
    assert SolverConfig.from_env().newton_precision == "bf16x3"
    with pytest.raises(ValueError):
        SolverConfig.from_env(newton_precision="fp16")
    monkeypatch.delenv("TDQ_NEWTON_PRECISION")
    tdq.set_seed(0)
    D = DomainND(["x", "t"], time_var="t")
    D.add("x", [-1.0, 1.0], 32)
    D.add("t", [0.0, 1.0], 16)
    D.generate_collocation_points(128)

    def f_model(u_model, x, t):
        u = u_model(torch.cat([x, t], 1))
        return tdq.grad(u, t) - 0.01 * tdq.grad(tdq.grad(u, x), x)

    m = tdq.CollocationSolverND(verbose=False)
    m.compile([2, 16, 16, 1], f_model, D, [dirichletBC(D, 0.0, "x", "upper")], device="cpu",
              precision="bf16", newton_precision="bf16x3")
    assert m.program().precision == "bf16"
    assert m._get_lbfgs_engine().program.precision == "bf16x3"
    assert m.program(precision="bf16") is m.program()   # same-precision request -> same program
    m.fit(tf_iter=3, newton_iter=3)
    assert math.isfinite(m.losses[-1]["Total Loss"])


def test_metrics_jsonl(tmp_path):
    from tensordiffeq_amd.boundaries import DomainND, dirichletBC
    tdq.set_seed(0)
    D = DomainND(["x", "t"], time_var="t")
    D.add("x", [-1.0, 1.0], 32)
    D.add("t", [0.0, 1.0], 16)
    D.generate_collocation_points(256)

    def f_model(u_model, x, t):
        u = u_model(torch.cat([x, t], 1))
        return tdq.grad(u, t) - 0.01 * tdq.grad(tdq.grad(u, x), x)

    m = tdq.CollocationSolverND(verbose=False)
    path = tmp_path / "m.jsonl"
    m.compile([2, 16, 16, 1], f_model, D, [dirichletBC(D, 0.0, "x", "upper")], device="cpu",
              metrics_path=str(path), log_every=5)
    m.fit(tf_iter=10, newton_iter=5)
    m.metrics.close()
    recs = read_jsonl(path)
    adam = [r for r in recs if r.get("phase") == "adam"]
    assert [r["epoch"] for r in adam] == [5, 10]
    assert set(adam[-1]["terms"]) == {t.name for t in m.program().terms}
    assert adam[-1]["pts_per_s"] > 0 and math.isfinite(adam[-1]["loss"])
    assert any(r.get("phase") == "lbfgs" for r in recs)
    assert np.isclose(adam[-1]["loss"], m.losses[9]["Total Loss"], rtol=1e-6)
    stop = [r for r in recs if r.get("event") == "lbfgs_stop"]
    assert len(stop) == 1 and stop[0]["n_iter"] <= 5 and stop[0]["reason"]
    assert m.fit_info["lbfgs"]["reason"] == stop[0]["reason"] and m.fit_info["adam"]["steps"] == 10


def test_kernel_profile_writes_trace_and_table(tmp_path, monkeypatch):
    """TDQ_PROFILE wraps fit() in torch.profiler: a Chrome trace and a kernel table per run."""
    from tests.test_solver import compiled
    from tensordiffeq_amd import profiling
    monkeypatch.setenv("TDQ_PROFILE", str(tmp_path / "prof"))
    monkeypatch.setattr(profiling, "_FIT_CALLS", [0])
    m = compiled("jet")
    m.fit(tf_iter=3)
    m.fit(tf_iter=2)   # a second fit keeps its own trace / table
    for k, n in ((0, 3), (1, 2)):
        trace = tmp_path / "prof" / f"fit_{k}" / "trace.json"
        table = tmp_path / "prof" / f"fit_{k}" / "kernels.txt"
        assert trace.exists() and trace.stat().st_size > 0
        lines = table.read_text().splitlines()
        assert lines[0].startswith(f"# CollocationSolverND.fit(tf_iter={n}")
        assert len(lines) > 3 and "%" in lines[2]


def test_adam_nan_raises_with_epoch():
    """Failure detection: a non-finite loss in the (device-history) Adam loop raises
    FloatingPointError naming the epoch instead of training on silently."""
    import pytest
    import torch
    from tests.test_solver import compiled
    m = compiled("jet")
    m.fit(tf_iter=3)
    with torch.no_grad():
        m.u_model.flat[5] = float("nan")
    with pytest.raises(FloatingPointError, match="epoch 3"):
        m.fit(tf_iter=4)


def test_stale_library_hash_is_refused(monkeypatch):
    """The loader refuses a libtdq_hip.so whose embedded source hash differs from csrc/."""
    import pytest
    from tensordiffeq_amd.ops import _lib
    if not __import__("os").path.exists(_lib.LIB_PATH):
        pytest.skip("library not built")
    lib = _lib.load()
    assert _lib.library_hash(lib) == _lib.expected_hash()
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "_err", None)
    monkeypatch.setattr(_lib, "expected_hash", lambda: "0000000000000000")
    with pytest.raises(_lib.NativeUnavailable, match="stale"):
        _lib.load(required=True)
    monkeypatch.setenv("TDQ_SKIP_HASH_CHECK", "1")
    monkeypatch.setattr(_lib, "_err", None)
    assert _lib.load(required=True) is not None


def test_lint_subset_clean():
    """The reference CI's flake8 subset (E9, F63, F7, F82 - tools/lint.py) over the whole repo."""
    import importlib.util
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("tdq_lint", os.path.join(root, "tools", "lint.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert mod.main([]) == 0
