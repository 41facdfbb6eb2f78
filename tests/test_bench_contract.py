"""bench.py's driver contract on CPU: one JSON line from rank 0 with the metric / config of
BASELINE.json, single process and 2 ranks over gloo (torchrun, 127.0.0.1) - the multi-rank path
includes the collective warm-up stop (a rank-local clock once let ranks run different numbers of
DP steps)."""
import json
import math
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = ["metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"]
SMALL = ["--steps", "3", "--warmup", "1", "--npts", "512", "--no-l2", "--min-warmup-s", "0.05"]


def _free_port():
    from tensordiffeq_amd.parallel.dist import free_port
    return free_port()


def _env():
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env.pop("WORLD_SIZE", None)
    env.pop("PYTEST_CURRENT_TEST", None)   # the scripts run as plain programs, not under pytest
    env["CUDA_VISIBLE_DEVICES"] = ""
    return env


def _last_json(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out[-2000:]
    return json.loads(lines[0])


def _check(rec, n):
    for k in KEYS:
        assert k in rec, k
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        assert rec["metric"] == json.load(f)["metric"]
    assert rec["n_gpus"] == n and rec["steps"] == 3 and rec["warmup"] == 1
    assert rec["value"] > 0 and rec["ms_per_step"] > 0 and rec["higher_is_better"] is True
    assert rec["config"]["global_batch"] == 512 * n and rec["config"]["parallelism"] == f"dp{n}"
    assert abs(rec["value"] - 512 * n / (rec["ms_per_step"] / 1000.0)) / rec["value"] < 1e-6


@pytest.mark.timeout(300)
def test_bench_single_process_json():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + SMALL, capture_output=True, text=True,
                       env=_env(), timeout=280, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    _check(_last_json(r.stdout), 1)


@pytest.mark.timeout(300)
def test_bench_two_ranks_gloo_json():
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--gpus", "2"] + SMALL
    r = subprocess.run(cmd, capture_output=True, text=True, env=_env(), timeout=280, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _last_json(r.stdout)
    _check(rec, 2)
    assert rec["allreduce"]["impl"] == "torch.distributed"     # CPU ranks: no peer all-reduce


@pytest.mark.timeout(300)
def test_bench_self_launch_two_ranks_json():
    """``python bench.py --gpus 2`` with no launcher: bench.py re-runs itself as 2 ranks (child
    processes under torch.distributed.run) and relays rank 0's single JSON line."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + SMALL, capture_output=True,
                       text=True, env=_env(), timeout=280, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _last_json(r.stdout)
    _check(rec, 2)
    assert rec["rank_ms_per_step"]["min"] <= rec["rank_ms_per_step"]["max"]
    assert rec["allreduce"]["replay"]["us_per_call"] > 0
    assert rec["allreduce"]["replay"]["mode"] == "host-launched"    # gloo keeps it out of graphs


SCRIPT_DIST = r'''
import os, sys, json
import numpy as np, torch
import tensordiffeq_amd as tdq
from tensordiffeq_amd.boundaries import DomainND, dirichletBC
D = DomainND(["x", "t"], time_var="t")
D.add("x", [-1.0, 1.0], 16); D.add("t", [0.0, 1.0], 8)
tdq.set_seed(0)
D.generate_collocation_points(256)
def f_model(u_model, x, t):
    u = u_model(torch.cat([x, t], 1))
    return tdq.grad(u, t) - 0.1 * tdq.grad(tdq.grad(u, x), x)
bcs = [dirichletBC(D, val=0.0, var="x", target="upper")]
m = tdq.CollocationSolverND(verbose=False)
m.compile([2, 8, 8, 1], f_model, D, bcs, dist=True, seed=0)
m.fit(tf_iter=3)
ctx = m.dist_ctx
with open(os.path.join(os.environ["OUT_DIR"], f"rank{ctx.rank}.json"), "w") as f:
    json.dump({"rank": ctx.rank, "world": ctx.world, "dist": ctx.is_distributed,
               "loss": m.losses[-1]["Total Loss"]}, f)
'''


@pytest.mark.timeout(300)
def test_compile_dist_true_self_launches(tmp_path):
    """Reference semantics (models.py:230-243, MirroredStrategy): ``compile(dist=True)`` in a plain
    ``python`` process trains on every visible device.  Here the script is re-run as one rank per
    device; TDQ_DIST_NPROC stands in for two visible devices on the CPU."""
    p = tmp_path / "dist_script.py"
    p.write_text(SCRIPT_DIST)
    env = _env()
    env["TDQ_DIST_NPROC"] = "2"
    env["OUT_DIR"] = str(tmp_path)
    r = subprocess.run([sys.executable, str(p)], capture_output=True, text=True, env=env, timeout=280, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    recs = [json.loads(q.read_text()) for q in sorted(tmp_path.glob("rank*.json"))]
    assert sorted(x["rank"] for x in recs) == [0, 1], r.stdout
    assert all(x["world"] == 2 and x["dist"] for x in recs)
    assert recs[0]["loss"] == pytest.approx(recs[1]["loss"], rel=1e-6)


@pytest.mark.timeout(300)
def test_compile_dist_true_one_device_warns(tmp_path):
    """With one (here: no) visible device and no launcher, dist=True says that it trains at world 1."""
    p = tmp_path / "dist_script.py"
    p.write_text(SCRIPT_DIST)
    env = _env()
    env["OUT_DIR"] = str(tmp_path)
    r = subprocess.run([sys.executable, str(p)], capture_output=True, text=True, env=env, timeout=280, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "training at world 1" in r.stderr
    recs = [json.loads(q.read_text()) for q in sorted(tmp_path.glob("rank*.json"))]
    assert len(recs) == 1 and recs[0]["world"] == 1 and not recs[0]["dist"]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("problem", ["ac-sa", "ac-dist"])
def test_bench_accuracy_under_dp_two_ranks(problem):
    """at --gpus N the accuracy schedule runs under data parallelism (points and
    SA weights sharded) and rank 0's JSON carries its L2 next to the throughput (tiny CPU sizes)."""
    args = ["--steps", "2", "--warmup", "1", "--min-warmup-s", "0.01", "--problem", problem, "--gpus", "2",
            "--acc-seeds", "0", "--acc-iters", "3", "--acc-newton", "3", "--acc-npts", "512"]
    args += ["--npts", "256"] if problem == "ac-sa" else ["--global-npts", "512"]
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       env=_env(), timeout=280, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _last_json(r.stdout)
    assert rec["n_gpus"] == 2
    assert rec["l2_full_schedule"] is not None and math.isfinite(rec["l2_full_schedule"]), rec
    assert "on 2 GPUs" in rec["accuracy_schedule"]
    assert len(rec["time_to_solution_s"]) == 1


@pytest.mark.timeout(300)
@pytest.mark.parametrize("how", ["ipykernel", "python-c", "slurm"])
def test_dist_true_never_relaunches_non_scripts(how, tmp_path):
    """a notebook kernel (argv[0] = ipykernel_launcher.py), ``python -c`` and a task that
    a non-torchrun launcher (srun) already started must train at world 1 instead of re-running
    something N times."""
    env = _env()
    env["TDQ_DIST_NPROC"] = "2"
    env["OUT_DIR"] = str(tmp_path)
    if how == "ipykernel":
        p = tmp_path / "ipykernel_launcher.py"
        p.write_text("import sys, types\nsys.modules['ipykernel'] = types.ModuleType('ipykernel')\n" + SCRIPT_DIST)
        cmd = [sys.executable, str(p)]
    elif how == "python-c":
        cmd = [sys.executable, "-c", SCRIPT_DIST]
    else:
        p = tmp_path / "dist_script.py"
        p.write_text(SCRIPT_DIST)
        env["SLURM_PROCID"] = "0"
        cmd = [sys.executable, str(p)]
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=280, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "launching 2 ranks" not in r.stderr
    recs = [json.loads(q.read_text()) for q in sorted(tmp_path.glob("rank*.json"))]
    assert len(recs) == 1 and recs[0]["world"] == 1


def test_relaunch_argv_forms(monkeypatch):
    import types
    from tensordiffeq_amd.parallel import dist as tdist
    main = types.ModuleType("__main__")
    main.__file__ = os.path.join(ROOT, "bench.py")
    main.__spec__ = None
    monkeypatch.setitem(sys.modules, "__main__", main)
    monkeypatch.setattr(sys, "argv", [os.path.join(ROOT, "bench.py"), "--gpus", "2"])
    monkeypatch.delitem(sys.modules, "ipykernel", raising=False)
    monkeypatch.delitem(sys.modules, "IPython", raising=False)
    assert tdist.relaunch_argv() == [os.path.join(ROOT, "bench.py"), "--gpus", "2"]
    # a library that imports IPython does not make a plain script interactive
    fake_ip = types.ModuleType("IPython")
    fake_ip.get_ipython = lambda: None
    monkeypatch.setitem(sys.modules, "IPython", fake_ip)
    assert tdist.relaunch_argv() == [os.path.join(ROOT, "bench.py"), "--gpus", "2"]
    fake_ip.get_ipython = lambda: object()                               # a running IPython shell
    assert tdist.relaunch_argv() is None
    monkeypatch.delitem(sys.modules, "IPython", raising=False)
    main.__spec__ = types.SimpleNamespace(name="examples.ac_dist")       # python -m examples.ac_dist
    assert tdist.relaunch_argv() == ["-m", "examples.ac_dist", "--gpus", "2"]
    main.__spec__ = None
    monkeypatch.setattr(sys, "argv", ["/elsewhere/ipykernel_launcher.py", "-f", "kernel.json"])
    assert tdist.relaunch_argv() is None                                  # __main__ is not argv[0]


PROBLEM_ARGS = {"ac-sa": ["--npts", "256"], "ac-baseline": ["--npts", "256"], "poisson": ["--npts", "256"],
                "ac-dist": ["--global-npts", "512"], "discovery": ["--global-npts", "512"]}


@pytest.mark.timeout(300)
@pytest.mark.parametrize("n", [1, 2])
@pytest.mark.parametrize("problem", sorted(PROBLEM_ARGS))
def test_bench_problems_json(problem, n):
    """Every BASELINE.json config through the same bench contract, single process and 2 gloo ranks
    (self-launched): one JSON line, the problem's scaling mode and point count."""
    args = ["--steps", "2", "--warmup", "1", "--no-l2", "--min-warmup-s", "0.01", "--problem", problem,
            "--gpus", str(n)] + PROBLEM_ARGS[problem]
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       env=_env(), timeout=280, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _last_json(r.stdout)
    assert rec["n_gpus"] == n and rec["config"]["problem"] == problem and rec["value"] > 0
    strong = "--global-npts" in PROBLEM_ARGS[problem]
    assert rec["scaling"] == ("strong" if strong else "weak")
    assert rec["config"]["global_batch"] == (512 if strong else 256 * n)
    assert rec["config"]["parallelism"] == f"dp{n}"
    if problem == "discovery":
        assert rec["unit"] == "data-pts/s"
