"""Data parallelism on the GPU path: 2 ranks share cuda:0 over gloo (RCCL refuses two ranks on one
device; a real multi-GPU RCCL run needs an 8-GPU node, which only the round-end driver gets).

Exercises everything the torchrun/RCCL benchmark runs except RCCL itself: HIP jet kernels + fused
loss on per-rank shards, SA weights sharded with the points, the HIP-graph capture split around the
flat-bucket all-reduce, and L-BFGS under DP.  Compared against a single-process full-batch run.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

import tensordiffeq_amd as tdq

pytestmark = pytest.mark.gpu
N_F = 4096


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _build(dist, world=1, precision=None):
    import bench
    return bench.build_problem(N_F // world, world, "hip", torch.device("cuda", 0), dist, precision)


def _worker(rank, world, port, q, precision):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from tensordiffeq_amd.parallel import dist as pdist
    pdist.reset_context()
    ctx = pdist.init_distributed(backend="gloo", device="cuda:0")
    m = _build(True, world, precision)
    assert m.active_backend == "hip"
    eng = m._get_engine(None, 10)
    loss, grads, terms = eng._phase_a()
    loss, grads, terms = eng._reduce(loss, grads, terms)
    res = {"loss": float(loss), "gflat": grads[0].detach().cpu().clone()}
    m.fit(tf_iter=8)                       # graph-captured (split around the all-reduce)
    res["hist"] = [h["Total Loss"] for h in m.losses]
    res["flat_after"] = m.u_model.flat.detach().cpu().clone()
    m.fit(newton_iter=3)
    res["lbfgs_loss"] = float(m.min_loss["l-bfgs"])
    if rank == 0:
        q.put(res)
    ctx.barrier()
    pdist.destroy()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("precision", ["bf16x3", "bf16"])
def test_dp_two_ranks_on_gpu_match_single_process(precision):
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
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, precision)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=500)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert res["loss"] == pytest.approx(loss, rel=1e-4)
    assert ((res["gflat"] - g_ref).norm() / g_ref.norm()).item() < 1e-3
    assert res["hist"] == pytest.approx(ref_hist, rel=1e-3)
    assert ((res["flat_after"] - ref_flat).norm() / ref_flat.norm()).item() < 1e-3
    assert res["lbfgs_loss"] == pytest.approx(float(ref.min_loss["l-bfgs"]), rel=5e-2)
