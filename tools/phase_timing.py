"""Per-phase timing of the split-bf16 (bf16x3 / bf16: --prec) jet kernels (WT = 8 instantiations) from in-kernel s_memtime stamps.

Builds ``csrc/build_timing/libtdq_hip_timing.so`` with ``-DTDQ_PHASE_TIMING`` (separate from the
production library), runs forward + backward of the Allen-Cahn plan on ``--npts`` points and prints,
for every stamp pair, the mean / median cycles per wave.  GPU only.
"""
import argparse
import ctypes
import glob
import os
import subprocess
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
CSRC = os.path.join(ROOT, "tensordiffeq_amd", "csrc")


def build():
    from tensordiffeq_amd.csrc import build as B
    out_dir = os.path.join(CSRC, "build_timing")
    os.makedirs(out_dir, exist_ok=True)
    objs = []
    for src in sorted(glob.glob(os.path.join(CSRC, "*.hip"))):
        obj = os.path.join(out_dir, os.path.basename(src) + ".o")
        cmd = [B.hipcc()] + B._flags() + ["-DTDQ_PHASE_TIMING", "-c", src, "-o", obj]
        subprocess.run(cmd, check=True)
        objs.append(obj)
    lib = os.path.join(out_dir, "libtdq_hip_timing.so")
    subprocess.run([B.hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", lib] + objs, check=True)
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--npts", type=int, default=50000)
    ap.add_argument("--lib", default=None)
    ap.add_argument("--prec", default="bf16x3", choices=["bf16x3", "bf16"])
    args = ap.parse_args()
    libpath = args.lib or build()
    from tensordiffeq_amd.ops import _lib
    lib = ctypes.CDLL(libpath)
    _lib._declare(lib)
    lib.tdq_set_timing_buffer.argtypes = [ctypes.c_void_p]
    from tensordiffeq_amd.jet import JetPlan
    from tensordiffeq_amd.models.networks import TanhMLP
    from tensordiffeq_amd.ops.jet_hip import stream_spec
    torch.manual_seed(0)
    N = args.npts
    net = TanhMLP([2, 128, 128, 128, 128, 1], device="cuda")
    X = (torch.rand(N, 2, device="cuda") * 2 - 1).contiguous()
    plan = JetPlan([(0,), (1,), (0, 0)], 2)
    spec = stream_spec(plan)
    spec_c = (ctypes.c_int * len(spec))(*spec)
    S = plan.S
    nwg = (N + 63) // 64
    ts = torch.zeros(nwg * 4 * 64, dtype=torch.int64, device="cuda")
    lib.tdq_set_timing_buffer(ts.data_ptr())
    J = torch.empty(S, N, 1, device="cuda")
    scr = torch.empty(lib.tdq_jet_bf3_scratch_floats(N, 2, (ctypes.c_int * 4)(128, 128, 128, 128), 4, S, 1), device="cuda")
    work = torch.empty(lib.tdq_jet_bf3_slab_floats(N, 2, (ctypes.c_int * 4)(128, 128, 128, 128), 1, 4), device="cuda")
    grad = torch.empty_like(net.flat)
    dJ = torch.randn(S, N, 1, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    P = net.flat.detach()
    lo = 1 if args.prec == "bf16x3" else 0
    for kind in ("fwd", "bwd"):
        for rep in range(3):
            ts.zero_()
            if kind == "fwd":
                rc = lib.tdq_jet_fwd_bf3(X.data_ptr(), P.data_ptr(), J.data_ptr(), scr.data_ptr(), N, 2, 128, 1, 4, S,
                                         spec_c, lo, st)
            else:
                rc = lib.tdq_jet_bwd_bf3(X.data_ptr(), P.data_ptr(), dJ.data_ptr(), scr.data_ptr(), work.data_ptr(),
                                         grad.data_ptr(), N, 2, 128, 1, 4, S, spec_c, lo, st)
            assert rc == 0, rc
            torch.cuda.synchronize()
        T = ts.view(nwg * 4, 64).cpu().numpy().astype(np.int64)
        used = [k for k in range(64) if (T[:, k] != 0).all()]
        print(f"== {kind}: stamps {used}; wave lifetime median {np.median(T[:, used[-1]] - T[:, used[0]]):.0f} cyc")
        for a, b in zip(used[:-1], used[1:]):
            d = T[:, b] - T[:, a]
            print(f"  {a:2d} -> {b:2d}: mean {d.mean():9.0f}  median {np.median(d):9.0f}  p90 {np.percentile(d, 90):9.0f}")
        start = T[:, used[0]]
        print(f"  kernel span {start.max() - start.min() + np.median(T[:, used[-1]] - start):.0f} cyc (approx)")


if __name__ == "__main__":
    main()
