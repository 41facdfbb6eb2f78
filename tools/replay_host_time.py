"""Is the AC-SA step host-bound?  Host enqueue time of the K-step graph replays vs their GPU time,
and the GPU time per step when the queue is pre-filled behind a spin kernel (the host cannot
starve the GPU then).  GPU only."""
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    import bench
    dev = torch.device("cuda", 0)
    m = bench.build_problem(50000, 1, "hip", dev, False, "bf16")
    eng = bench.get_engine(m, 2000)
    eng.run(300)
    torch.cuda.synchronize()
    K = eng._unroll()
    R = 40
    eng._ensure_hist(R * K * 4 + 10)
    g = eng.graph_k
    # 1) plain: host enqueue time and wall per step
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(R):
        g.replay()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"K={K} replays={R}: host enqueue {1e6 * (t1 - t0) / (R * K):.1f} us/step, wall {1e6 * (t2 - t0) / (R * K):.1f} us/step")
    # 2) pre-filled queue: a spin kernel first, then every replay enqueued behind it
    for spin in (20_000_000, 50_000_000):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        torch.cuda._sleep(spin)
        e0.record()
        t0 = time.perf_counter()
        for _ in range(R):
            g.replay()
        t1 = time.perf_counter()
        e1.record()
        torch.cuda.synchronize()
        print(f"spin {spin}: enqueue {1e6 * (t1 - t0) / (R * K):.1f} us/step (host), GPU {1e3 * e0.elapsed_time(e1) / (R * K):.1f} us/step")
    # 3) events around the plain loop
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(R):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    print(f"plain events: GPU {1e3 * e0.elapsed_time(e1) / (R * K):.1f} us/step")


if __name__ == "__main__":
    main()
