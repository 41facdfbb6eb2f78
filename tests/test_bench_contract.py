"""bench.py's driver contract on CPU: one JSON line from rank 0 with the metric / config of
BASELINE.json, single process and 2 ranks over gloo (torchrun, 127.0.0.1) - the multi-rank path
includes the collective warm-up stop (a rank-local clock once let ranks run different numbers of
DP steps)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = ["metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"]
SMALL = ["--steps", "3", "--warmup", "1", "--npts", "512", "--no-l2", "--min-warmup-s", "0.05"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _env():
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env.pop("WORLD_SIZE", None)
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
