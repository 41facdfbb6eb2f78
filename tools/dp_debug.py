"""Per-rank loss/term dump for the 2-ranks-on-one-GPU DP check (diagnostic)."""
import os, sys, socket
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.multiprocessing as mp
N_F = 4096


def build(dist, world, backend):
    import bench
    return bench.build_problem(N_F, world, backend, torch.device("cuda", 0), dist)


def worker(rank, world, port, q, backend, fused):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), TDQ_FUSED_LOSS=fused)
    from tensordiffeq_amd.parallel import dist as pdist
    pdist.reset_context()
    ctx = pdist.init_distributed(backend="gloo", device="cuda:0")
    m = build(True, world, backend)
    prog = m.program()
    eng = m._get_engine(None, 10)
    loss, grads, terms = eng._phase_a()
    torch.cuda.synchronize()
    lloc = float(loss)
    tl = [float(t) for t in terms]
    loss, grads, terms = eng._reduce(loss, grads, terms)
    torch.cuda.synchronize()
    info = dict(rank=rank, local=lloc, local_terms=tl, reduced=float(loss), fused=prog.fused_op is not None,
                nloc=m.X_f_local.shape[0], denoms=[t.denom for t in prog.terms], scales=[t.scale for t in prog.terms],
                x0=m.X_f_local[:2].tolist(), lam0=m.lambdas[0][:3].flatten().tolist())
    q.put(info)
    ctx.barrier()
    pdist.destroy()


def main():
    for backend, fused in (("hip", "1"), ("hip", "0"), ("jet", "1")):
        os.environ["TDQ_FUSED_LOSS"] = fused
        ref = build(False, 1, backend)
        eng = ref._get_engine(None, 10)
        loss, grads, terms = eng._phase_a()
        print(f"== backend {backend} fused {fused}: single {float(loss):.6f} terms {[float(t) for t in terms]}",
              flush=True)
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
        ps = [ctx.Process(target=worker, args=(r, 2, port, q, backend, fused)) for r in range(2)]
        [p.start() for p in ps]
        for _ in range(2):
            print(q.get(timeout=300), flush=True)
        [p.join(timeout=60) for p in ps]


if __name__ == "__main__":
    main()
