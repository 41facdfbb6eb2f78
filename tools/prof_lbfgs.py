"""L-BFGS iteration profile target: the flagship AC-SA problem, a few Adam steps, then ``--iters``
device L-BFGS iterations in the L-BFGS precision (bf16x3).  Run under rocprofv3 --kernel-trace
--stats (tools/gpu_runs/r3_d.sh); prints the wall time per iteration."""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=500)
    ap.add_argument("--npts", type=int, default=50000)
    ap.add_argument("--ts", action="store_true",
                    help="phase stamps of the dots + logic kernel (TDQ_LBFGS_TS=1, lbfgs.hip LB_TS0)")
    a = ap.parse_args()
    if a.ts:
        os.environ["TDQ_LBFGS_TS"] = "1"
    import torch
    import bench
    m = bench.build_problem(a.npts, 1, "hip", torch.device("cuda", 0), False, "bf16", newton_precision="bf16x3")
    m.fit(tf_iter=3000)     # a trained start: L-BFGS's fixed step diverges from a raw init
    m.fit(newton_iter=20)   # capture + warm
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    m.fit(newton_iter=a.iters)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    info = m.fit_info["lbfgs"]
    ht = getattr(m.lbfgs_state, "host_times", None)
    if ht and ht["batches"]:
        print(json.dumps({"host_enqueue_s": ht["enqueue_s"], "host_wait_s": ht["wait_s"], "batches": ht["batches"]}))
    if a.ts:   # 100 MHz real-time counter ticks summed over the iterations that ran the full logic
        st = m.lbfgs_state.st.cpu().tolist()
        n = max(1.0, st[23])
        ticks = st[20] + st[21] + st[22]
        print(json.dumps({"ts_iters": st[23], "shader_clock_mhz": 100.0 * st[19] / max(ticks, 1.0),
                          "us_step1_loads": st[20] / n / 100, "us_step2_3_tests": st[21] / n / 100,
                          "us_step4_5_solves": st[22] / n / 100}))
    print(json.dumps({"iters": info["n_iter"], "reason": info["reason"], "wall_s": dt,
                      "ms_per_iter": 1e3 * dt / max(1, info["n_iter"]),
                      "fused_update": os.environ.get("TDQ_LBFGS_FUSED", "1")}))


if __name__ == "__main__":
    main()
