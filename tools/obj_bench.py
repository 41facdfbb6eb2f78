"""Time the L-BFGS objective ``[grad | loss]`` (LossGradEngine.evaluate_fg) of AC-SA in one
precision - the one-launch fused objective or, with TDQ_FUSED_STEP=0, the separate launches:

    python tools/obj_bench.py --precision bf16x3 --reps 300

Prints one JSON line (us per evaluation, back-to-back eager launches, after a warm-up)."""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from tensordiffeq_amd.fit import LossGradEngine
    from tensordiffeq_amd.ops import fused_step
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="bf16x3")
    ap.add_argument("--npts", type=int, default=50000)
    ap.add_argument("--reps", type=int, default=300)
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    m = bench.build_problem(a.npts, 1, "hip", torch.device("cuda", 0), False, a.precision)
    prog = m.program()
    fs = fused_step.for_program(prog)
    eng = LossGradEngine(m, prog, m.lambdas)
    for _ in range(20):
        fg = eng.evaluate_fg()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        fg = eng.evaluate_fg()
    e1.record()
    torch.cuda.synchronize()
    us = 1e3 * e0.elapsed_time(e1) / a.reps
    print(json.dumps({"tag": a.tag, "precision": a.precision, "npts": a.npts, "fused": fs is not None,
                      "defines": os.environ.get("TDQ_FUSED_STEP_DEFINES", ""), "us_per_eval": round(us, 2),
                      "loss": float(fg[-1])}))


if __name__ == "__main__":
    main()
