"""Per-phase cycles of the persistent jet kernels (csrc/jet_fused.h, LM = 3 instantiations) from
in-kernel s_memtime stamps of the first tile of every workgroup.

Builds ``csrc/build_timing_fz/libtdq_hip.so`` with ``-DTDQ_PHASE_TIMING`` (a separate library),
runs the forward and the recompute backward of the Allen-Cahn plan on ``--npts`` points and prints
the median cycles per wave between consecutive stamps.  GPU only.
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

NAMES = {0: "start", 1: "tile loads", 2: "layer 0", 3: "gemm 1", 4: "epi 1", 5: "gemm 2", 6: "epi 2",
         7: "gemm 3", 8: "epi 3 (+out bwd)", 62: "all tiles", 63: "slab row"}
for k, ly in enumerate((3, 2, 1)):
    b = 10 + 5 * k
    NAMES.update({b: f"gemm K_{ly}", b + 1: f"adjoint + dK_{ly}", b + 2: f"barrier {ly}", b + 3: f"write zb {ly}",
                  b + 4: f"rebuild/barrier {ly}"})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--npts", type=int, default=50000)
    a = ap.parse_args()
    os.environ["TDQ_FUSED"] = "1"
    from tensordiffeq_amd.csrc import build as B
    lib_path = B.build(variant="timing_fz", defines=("TDQ_PHASE_TIMING",), verbose=False)
    os.environ["TDQ_LIB_PATH"] = lib_path
    from tensordiffeq_amd.ops import _lib, jet_hip
    _lib.LIB_PATH = lib_path
    lib = _lib.load(required=True)
    lib.tdq_fz_set_timing_buffer.argtypes = [ctypes.c_void_p]
    from tensordiffeq_amd.jet import JetPlan
    from tensordiffeq_amd.models.networks import TanhMLP
    torch.manual_seed(0)
    N = a.npts
    net = TanhMLP([2, 128, 128, 128, 128, 1], device="cuda")
    X = (torch.rand(N, 2, device="cuda") * 2 - 1).contiguous()
    plan = JetPlan([(0,), (1,), (0, 0)], 2)
    G = lib.tdq_jet_fused_rows(N)
    ts = torch.zeros(G * 8 * 64, dtype=torch.int64, device="cuda")
    lib.tdq_fz_set_timing_buffer(ctypes.c_void_p(ts.data_ptr()))
    p = net.flat.detach().clone().requires_grad_(True)
    for it in range(3):
        ts.zero_()
        J = jet_hip.JetMLPFunction.apply(X, p, net, plan, "bf16")
        J.sum().backward()
        torch.cuda.synchronize()
    t = ts.view(G * 8, 64).cpu().numpy().astype(np.float64)
    ks = [k for k in sorted(NAMES) if (t[:, k] != 0).any()]
    print(f"# persistent backward (last launch) on {N} points, {G} workgroups x 8 waves; cycles per wave")
    print("# phase                      median      p90")
    prev = ks[0]
    for k in ks[1:]:
        d = t[:, k] - t[:, prev]
        d = d[(t[:, k] != 0) & (t[:, prev] != 0)]
        print(f"  {NAMES.get(k, k):24s} {np.median(d):9.0f} {np.percentile(d, 90):9.0f}")
        prev = k
    tot = t[:, 62] - t[:, 0]
    print(f"  {'tile loop total':24s} {np.median(tot):9.0f} {np.percentile(tot, 90):9.0f}")


if __name__ == "__main__":
    main()
