"""One-shot peer-memory all-reduce (csrc/peer.hip, parallel/peer.py) with 2 and 4 ranks sharing cuda:0.

Several processes on one GPU exercise everything the 8-GPU xGMI path runs except the fabric: the
uncached IPC-shared receive slots and flags, the push / flag / bounded wait / rank-order sum
kernel, the self-test and selection at start-up, graph capture of the kernel, and both receive
parities.  The control plane (IPC handle exchange) rides on a gloo group.
"""
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

SIZES = [1, 3, 1000, 1024, 1025, 4097, 49_408, 200_001]


def _free_port():
    from tensordiffeq_amd.parallel.dist import free_port
    return free_port()


def _guard(fn, rank, world, port, q):
    """A failing rank reports its traceback at once (the parent then stops every rank and fails)
    instead of leaving the others waiting in the rendezvous."""
    try:
        fn(rank, world, port, q)
    except BaseException:  # noqa: BLE001 - reported to the parent, then re-raised
        import traceback
        q.put((rank, {"error": traceback.format_exc()}))
        raise


def _collect(procs, q, timeout):
    got = {}
    for _ in procs:
        r, res = q.get(timeout=timeout)
        if "error" in res:
            for p in procs:   # exactly the processes this test started
                if p.is_alive():
                    p.kill()
            pytest.fail(f"rank {r} failed:\n{res['error']}")
        got[r] = res
    return got


def _worker_body(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), TDQ_PEER_ALLREDUCE="1", TDQ_PEER_TIMEOUT_S="20")
    from tensordiffeq_amd.parallel import dist as pdist
    pdist.reset_context()
    ctx = pdist.init_distributed(backend="gloo", device="cuda:0")
    res = {"info": dict(ctx.allreduce_info), "on": ctx.peer is not None}
    if ctx.peer is not None:
        dev = ctx.device
        outs = {}
        for n in SIZES:
            g = torch.Generator().manual_seed(1000 * n + rank)
            x = torch.randn(n, generator=g)
            buf = x.to(dev)
            ctx.all_reduce_(buf)
            outs[n] = buf.cpu().numpy().copy()
        # captured: 4 all-reduces in one graph, replayed 3 times (the call counters advance on the
        # device, so every replay is a new pair of calls)
        n = 49_408
        static = torch.zeros(n, device=dev)
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                for _ in range(4):
                    static.mul_(0.5)
                    ctx.all_reduce_(static)
        torch.cuda.current_stream(dev).wait_stream(s)
        graph_out = []
        for rep in range(3):
            static.copy_(torch.full((n,), float(rank + 1 + rep), device=dev))
            g.replay()
            torch.cuda.synchronize(dev)
            graph_out.append(static.cpu().numpy().copy())
        ctx.check_health()
        res.update(outs=outs, graph=graph_out, err=int(ctx.peer.err.item()))
    q.put((rank, res))
    ctx.barrier()
    pdist.destroy()


def _worker(rank, world, port, q):
    _guard(_worker_body, rank, world, port, q)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 4])
def test_peer_allreduce_ranks_one_gpu(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = _collect(procs, q, 250)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    print("PEER", world, got[0]["info"])
    for r in range(world):
        assert got[r]["on"] and got[r]["err"] == 0, (r, got[r]["info"])
    for n in SIZES:
        want = torch.zeros(n)
        for r in range(world):                           # the kernel's order: rank 0, 1, ...
            want = want + torch.randn(n, generator=torch.Generator().manual_seed(1000 * n + r))
        for r in range(world):
            assert np.array_equal(got[r]["outs"][n], want.numpy()), (n, r)
    for rep in range(3):
        # halves of the start values summed, then each later call halves and re-sums S (x world / 2)
        v = 0.5 * sum(float(r + 1 + rep) for r in range(world)) * (0.5 * world) ** 3
        for r in range(world):
            assert np.all(got[r]["graph"][rep] == v), (rep, r)


def _timeout_worker_body(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), TDQ_PEER_ALLREDUCE="1", TDQ_PEER_TIMEOUT_S="2")
    from tensordiffeq_amd.parallel import dist as pdist
    pdist.reset_context()
    ctx = pdist.init_distributed(backend="gloo", device="cuda:0")
    res = {"on": ctx.peer is not None}
    if ctx.peer is not None:
        buf = torch.ones(4096, device=ctx.device)
        if rank == 0:            # rank 1 skips this call: rank 0's waits must time out, not hang
            ctx.all_reduce_(buf)
        torch.cuda.synchronize()
        try:
            ctx.check_health()
            res["raised"] = False
        except RuntimeError as e:
            res["raised"] = "timed out" in str(e)
    q.put((rank, res))
    ctx.barrier()
    # the communicator's call counters now disagree: do not close through another collective
    ctx.peer = None
    pdist.destroy()


def _timeout_worker(rank, world, port, q):
    _guard(_timeout_worker_body, rank, world, port, q)


@pytest.mark.timeout(200)
def test_peer_allreduce_times_out_instead_of_hanging():
    """A rank that never arrives: the waiting rank's kernel gives up after TDQ_PEER_TIMEOUT_S, sets
    its error word and drains (the GPU is never held), and check_health() raises."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_timeout_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = _collect(procs, q, 150)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0]["on"] and got[1]["on"]
    assert got[0]["raised"] is True and got[1]["raised"] is False
