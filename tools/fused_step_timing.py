"""Per-phase cycles of the fused training step (ops/fused_step.py, csrc/jet_fused.h MODE 2) from
in-kernel s_memtime stamps of the first tile of every workgroup.

The run-time compiled kernel is built with ``-DTDQ_PHASE_TIMING`` (``TDQ_FUSED_STEP_TIMING=1``),
one AC-SA loss + gradient evaluation at ``--npts`` collocation points runs through the fused step,
and the median / p90 cycles per wave between consecutive stamps are printed.  GPU only.
"""
import argparse
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

NAMES = {0: "start", 1: "tile loads", 2: "layer 0", 3: "gemm 1", 4: "epi 1", 5: "gemm 2", 6: "epi 2",
         7: "gemm 3", 8: "epi 3 + out dots", 9: "loss (point-threads)", 62: "all tiles", 63: "slab row + partials"}
for k, ly in enumerate((3, 2, 1)):
    b = 10 + 5 * k
    NAMES.update({b: f"gemm K_{ly}" + (" (+ out bwd)" if ly == 3 else ""), b + 1: f"adjoint + dK_{ly}",
                  b + 2: f"barrier {ly}", b + 3: f"write zb {ly}", b + 4: f"rebuild/barrier {ly}"})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--npts", type=int, default=50000)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "bf16x3"],
                    help="bf16: the Adam step (32-point tiles); bf16x3: the L-BFGS objective (16-point tiles)")
    a = ap.parse_args()
    os.environ["TDQ_FUSED_STEP_TIMING"] = "1"
    import bench
    from tensordiffeq_amd.fit import LossGradEngine
    from tensordiffeq_amd.ops import fused_step
    m = bench.build_problem(a.npts, 1, "hip", torch.device("cuda", 0), False, a.precision)
    prog = m.program()
    fs = fused_step.for_program(prog)
    assert fs is not None, prog.fused_step_reason
    ts = torch.zeros(fs.G * 8 * 64, dtype=torch.int64, device="cuda")
    fs.set_timing_buffer(ts)
    eng = LossGradEngine(m, prog, m.lambdas)
    for _ in range(3):
        ts.zero_()
        eng.evaluate_fg()
        torch.cuda.synchronize()
    t = ts.view(fs.G * 8, 64).cpu().numpy().astype(np.float64)
    ks = [k for k in sorted(NAMES) if (t[:, k] != 0).any()]
    tile = os.environ.get("TDQ_FUSED_STEP_DEFINES", "")
    print(f"# fused step ({a.precision}) on {a.npts} residual points: {fs.G} workgroups x 8 waves, tiles of "
          f"{fs.pt} points; cycles per wave ({'tile t0 + 1' if 'FZ_TS_TILE=1' in tile else 'first tile'})")
    print("# phase                        median      p90")
    prev = ks[0]
    for k in ks[1:]:
        d = t[:, k] - t[:, prev]
        d = d[(t[:, k] != 0) & (t[:, prev] != 0)]
        print(f"  {NAMES.get(k, k):28s} {np.median(d):9.0f} {np.percentile(d, 90):9.0f}")
        prev = k
    tot = t[:, 62] - t[:, 0]
    ntl = -(-(fs.N - fs.p_lo) // fs.pt)
    print(f"  {'tile loop total':28s} {np.median(tot):9.0f} {np.percentile(tot, 90):9.0f}"
          f"   ({ntl} tiles over {fs.G} workgroups)")


if __name__ == "__main__":
    main()
