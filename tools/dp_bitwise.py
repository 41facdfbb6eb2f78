"""Forced DP at world 1 vs the single process, step by step (debug aid for
tests/test_dist_gpu.py::test_forced_dp_rccl_world1_matches_single_process): prints the Adam loss
history of both with full precision and the first step where they differ."""
import os
import sys

import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _build(dist, precision="bf16", n_f=4096):
    import bench
    return bench.build_problem(n_f, 1, "hip", torch.device("cuda", 0), dist, precision)


def worker(q, dp_graph, iters):
    sys.path.insert(0, ROOT)
    from tensordiffeq_amd.parallel import dist as pdist
    if dp_graph != "single":
        os.environ.update(TDQ_FORCE_DP="1", WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", TDQ_DP_GRAPH=dp_graph)
        os.environ.pop("MASTER_PORT", None)
        pdist.reset_context()
        pdist.init_distributed(device="cuda:0")
    m = _build(dp_graph != "single")
    flats = [m.u_model.flat.detach().cpu().clone()]
    for _ in range(iters):
        m.fit(tf_iter=1)
        flats.append(m.u_model.flat.detach().cpu().clone())
    q.put({"hist": [h["Total Loss"] for h in m.losses], "flats": [f.numpy() for f in flats]})
    if dp_graph != "single":
        pdist.destroy()


def main():
    iters = 8
    ref = _build(False)
    flats = [ref.u_model.flat.detach().cpu().clone()]
    for _ in range(iters):
        ref.fit(tf_iter=1)
        flats.append(ref.u_model.flat.detach().cpu().clone())
    hist = [h["Total Loss"] for h in ref.losses]
    for dp_graph in ("single", "1"):
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        p = ctx.Process(target=worker, args=(q, dp_graph, iters))
        p.start()
        res = q.get(timeout=300)
        p.join(timeout=60)
        print(f"dp_graph={dp_graph}")
        for k, (a, b) in enumerate(zip(hist, res["hist"])):
            print(f"  step {k}: single {a!r} dp {b!r} {'EQUAL' if a == b else 'DIFF'}")
        for k, (a, b) in enumerate(zip(flats, res["flats"])):
            d = (a - torch.from_numpy(b)).abs()
            print(f"  params after {k} steps: max |diff| {float(d.max()):.3e} at {int(d.argmax())} (of {a.numel()})")


if __name__ == "__main__":
    main()
