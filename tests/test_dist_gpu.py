"""Data parallelism on the GPU path: 2 ranks share cuda:0 over gloo (RCCL refuses two ranks on one
device; a real multi-GPU RCCL run needs an 8-GPU node, which only the round-end driver gets).

Exercises everything the torchrun/RCCL benchmark runs except RCCL itself: HIP jet kernels + fused
loss on per-rank shards, SA weights sharded with the points, the HIP-graph capture split around the
flat-bucket all-reduce, and L-BFGS under DP.  Compared against a single-process full-batch run.
"""
import os

import pytest
import torch
import torch.multiprocessing as mp

import tensordiffeq_amd as tdq

pytestmark = pytest.mark.gpu
N_F = 4096


def _free_port():
    from tensordiffeq_amd.parallel.dist import free_port
    return free_port()


def _build(dist, world=1, precision=None, n_f=N_F):
    import bench
    return bench.build_problem(n_f, world, "hip", torch.device("cuda", 0), dist, precision)


def _worker(rank, world, port, q, precision, peer="0"):
    """A failing rank reports its traceback at once (the parent stops both ranks and fails)
    instead of leaving the other waiting in a collective until the test's timeout."""
    try:
        _worker_body(rank, world, port, q, precision, peer)
    except BaseException:  # noqa: BLE001 - reported to the parent, then re-raised
        import traceback
        q.put({"error": f"rank {rank}: " + traceback.format_exc()})
        raise


def _worker_body(rank, world, port, q, precision, peer):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), TDQ_PEER_ALLREDUCE=peer,
                      TDQ_STEP_UNROLL="4")
    from tensordiffeq_amd.parallel import dist as pdist
    pdist.reset_context()
    ctx = pdist.init_distributed(backend="gloo", device="cuda:0")
    m = _build(True, world, precision)
    assert m.active_backend == "hip"
    eng = m._get_engine(None, 10)
    loss, grads, terms = eng._phase_a()
    loss, grads, terms = eng._reduce(loss, grads, terms)
    # numpy over the queue: a torch tensor travels as a shared-memory handle that is gone once
    # this process exits
    res = {"loss": float(loss), "gflat": grads[0].detach().cpu().numpy().copy()}
    m.fit(tf_iter=8)                       # graph-captured (split around the all-reduce)
    res["hist"] = [h["Total Loss"] for h in m.losses]
    res["peer"] = ctx.peer is not None
    res["one_graph"] = m._get_engine(None, 1).graph_b is None
    res["k_graph"] = getattr(m._get_engine(None, 1), "graph_k", None) is not None
    res["flat_after"] = m.u_model.flat.detach().cpu().numpy().copy()
    m.fit(newton_iter=3)
    res["lbfgs_loss"] = float(m.min_loss["l-bfgs"])
    if rank == 0:
        q.put(res)
    ctx.barrier()
    pdist.destroy()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("precision,peer", [("bf16x3", "0"), ("bf16", "0"), ("bf16", "1")])
def test_dp_two_ranks_on_gpu_match_single_process(precision, peer):
    """peer "1": the bucket all-reduce is the one-shot peer kernel (csrc/peer.hip), captured in the
    step graph (one replay per step); "0": gloo between two graphs."""
    ref = _build(False, 1, precision)
    eng = ref._get_engine(None, 10)
    loss, grads, terms = eng._phase_a()
    loss = float(loss)   # persistent device buffer: read before fit() overwrites it
    g_ref = grads[0].detach().cpu().clone()
    ref.fit(tf_iter=8)
    ref_hist = [h["Total Loss"] for h in ref.losses]
    ref_flat = ref.u_model.flat.detach().cpu().clone()
    ref.fit(newton_iter=3)

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, precision, peer)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=500)
    if "error" in res:
        for p in procs:   # exactly the processes this test started
            if p.is_alive():
                p.kill()
        pytest.fail(res["error"])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    # peer: the all-reduce is a graph node, so 4-step graphs run too (TDQ_STEP_UNROLL=4, 8 steps)
    assert res["peer"] == (peer == "1") and res["one_graph"] == (peer == "1") and res["k_graph"] == (peer == "1")
    assert res["loss"] == pytest.approx(loss, rel=1e-4)
    gflat, flat_after = torch.from_numpy(res["gflat"]), torch.from_numpy(res["flat_after"])
    assert ((gflat - g_ref).norm() / g_ref.norm()).item() < 1e-3
    assert res["hist"] == pytest.approx(ref_hist, rel=1e-3)
    assert ((flat_after - ref_flat).norm() / ref_flat.norm()).item() < 1e-3
    assert res["lbfgs_loss"] == pytest.approx(float(ref.min_loss["l-bfgs"]), rel=5e-2)


def _forced_worker(q, precision, dp_graph, n_f=N_F, split="auto", iters=8, unroll="8"):
    os.environ.update(TDQ_FORCE_DP="1", WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", TDQ_DP_GRAPH=dp_graph,
                      TDQ_SPLIT=split, TDQ_STEP_UNROLL=unroll)
    os.environ.pop("MASTER_PORT", None)
    from tensordiffeq_amd.parallel import dist as pdist
    pdist.reset_context()
    ctx = pdist.init_distributed(device="cuda:0")       # backend nccl = RCCL
    assert ctx.backend == "nccl" and ctx.is_distributed and ctx.forced
    assert ctx.graph_collectives == (dp_graph == "1")
    m = _build(True, 1, precision, n_f)
    assert m.active_backend == "hip"
    m.fit(tf_iter=iters)
    eng = m._get_engine(None, 1)
    res = {"hist": [h["Total Loss"] for h in m.losses], "flat": m.u_model.flat.detach().cpu().numpy().copy(),
           "one_graph": eng.graph_b is None, "ranges": getattr(eng, "_ranges", None),
           "k_graph": getattr(eng, "graph_k", None) is not None}
    m.fit(newton_iter=3)
    res["lbfgs_loss"] = float(m.min_loss["l-bfgs"])
    q.put(res)
    pdist.destroy()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("dp_graph", ["1", "0"])
def test_forced_dp_rccl_world1_matches_single_process(dp_graph):
    """RCCL on the one-GPU box: TDQ_FORCE_DP=1 builds a real nccl (RCCL) process group at world 1;
    the DP step (bucket all-reduce captured in the step graph, or launched between two graphs with
    TDQ_DP_GRAPH=0) and the DP L-BFGS reproduce the single-process trajectory."""
    precision = "bf16"
    ref = _build(False, 1, precision)
    ref.fit(tf_iter=8)
    ref_hist = [h["Total Loss"] for h in ref.losses]
    ref_flat = ref.u_model.flat.detach().cpu().clone()
    ref.fit(newton_iter=3)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_forced_worker, args=(q, precision, dp_graph))
    p.start()
    res = q.get(timeout=500)
    p.join(timeout=120)
    assert p.exitcode == 0
    assert res["one_graph"] == (dp_graph == "1")
    assert res["hist"] == pytest.approx(ref_hist, rel=1e-6)
    assert torch.allclose(torch.from_numpy(res["flat"]), ref_flat, rtol=1e-6, atol=1e-7)
    assert res["lbfgs_loss"] == pytest.approx(float(ref.min_loss["l-bfgs"]), rel=1e-6)


@pytest.mark.timeout(600)
def test_forced_dp_rccl_point_ranges(monkeypatch):
    """The DP step with its points in two ranges on concurrent graph branches (TDQ_SPLIT, the
    in-place bucket tail after them, RCCL all-reduce in the graph) against the single-process run
    with single launches."""
    precision, n_f = "bf16", 20000
    monkeypatch.setenv("TDQ_SPLIT", "0")
    monkeypatch.setenv("TDQ_FUSED_STEP", "0")   # point ranges serve the separate-launch step (inherited by the worker)
    ref = _build(False, 1, precision, n_f)
    ref.fit(tf_iter=8)
    ref_hist = [h["Total Loss"] for h in ref.losses]
    ref_flat = ref.u_model.flat.detach().cpu().clone()
    ref.fit(newton_iter=3)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_forced_worker, args=(q, precision, "1", n_f, "0.5"))
    p.start()
    res = q.get(timeout=500)
    p.join(timeout=120)
    assert p.exitcode == 0
    assert res["ranges"] is not None and len(res["ranges"]) == 2
    assert res["hist"] == pytest.approx(ref_hist, rel=1e-6)
    assert torch.allclose(torch.from_numpy(res["flat"]), ref_flat, rtol=1e-6, atol=1e-7)
    assert res["lbfgs_loss"] == pytest.approx(float(ref.min_loss["l-bfgs"]), rel=1e-6)


@pytest.mark.timeout(600)
def test_forced_dp_rccl_multistep_graph():
    """DP with the all-reduce in the graph also runs K steps per graph (TDQ_STEP_UNROLL): 4-step
    graphs over persistent step buffers, RCCL all-reduce inside, against the single process."""
    precision, iters = "bf16", 21
    ref = _build(False, 1, precision)
    ref.fit(tf_iter=iters)
    ref_hist = [h["Total Loss"] for h in ref.losses]
    ref_flat = ref.u_model.flat.detach().cpu().clone()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_forced_worker, args=(q, precision, "1", N_F, "auto", iters, "4"))
    p.start()
    res = q.get(timeout=500)
    p.join(timeout=120)
    assert p.exitcode == 0
    assert res["one_graph"] and res["k_graph"]
    assert res["hist"] == pytest.approx(ref_hist, rel=1e-6)
    assert torch.allclose(torch.from_numpy(res["flat"]), ref_flat, rtol=1e-6, atol=1e-7)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("problem", ["ac-sa", "ac-baseline"])
def test_bench_self_launch_two_ranks_share_gpu(problem):
    """``python bench.py --gpus 2`` with no launcher on the one-GPU box: bench.py starts the two ranks
    itself (children under torch.distributed.run); they share cuda:0 over gloo + the peer all-reduce
    (TDQ_DIST_BACKEND=gloo: RCCL refuses two ranks on one device) and rank 0 prints one JSON line
    with the per-rank step times and the in-graph all-reduce time."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(TDQ_DIST_BACKEND="gloo", PYTHONPATH=root + os.pathsep + env.get("PYTHONPATH", ""))
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "20", "--warmup", "4",
           "--npts", "8192", "--no-l2", "--min-warmup-s", "0.2", "--problem", problem]
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=280, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    rec = json.loads(lines[0])
    print("SELF_LAUNCH", problem, json.dumps({k: rec[k] for k in ("n_gpus", "ms_per_step", "rank_ms_per_step", "allreduce")}))
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2" and rec["config"]["backend"] == "hip"
    assert rec["rank_ms_per_step"]["min"] <= rec["rank_ms_per_step"]["max"]
    assert rec["allreduce"]["replay"]["us_per_call"] > 0
