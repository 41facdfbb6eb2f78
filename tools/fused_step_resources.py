"""Register / LDS / spill report of the generated fused-step kernels (bf16 step and bf16x3
objective) for the AC-SA program, compiled offline with hipcc for gfx950 (no GPU needed):

    python tools/fused_step_resources.py [--out DIR]

Prints hipcc's kernel-resource-usage remarks (VGPRs, AGPRs, spills, LDS, occupancy)."""
import argparse
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def sources():
    from tensordiffeq_amd import fusion
    from tensordiffeq_amd.ops import _lib, fused_step, jet_hip
    from tensordiffeq_amd.ops.jet_mlp import hip_config
    from tensordiffeq_amd.ops.loss_fused import FusedLossOp
    from tests.test_fused_step import _deep
    m = _deep("ac", [2, 128, 128, 128, 128, 1])
    prog = m.program()
    fl = fusion.build(prog, m.lambdas)
    op = FusedLossOp(fl, prog, m.lambdas, fusion.scalar_values(fl, m.lambdas, None), fl.lam_offsets)
    cfg = hip_config(prog.net, prog.plan, "bf16")
    lib = _lib.load()
    spec = jet_hip.stream_spec(prog.plan)
    S = cfg["S"]
    nso = sum(1 for s in range(S) if spec[3 * s] == 2)
    layout, pos = [], 0
    for gr in fl.groups:
        ns = len(gr.segs)
        pos += pos % 2 if ns == 2 else 0
        layout.append((gr.program, pos, ns, gr.n))
        pos += ns * gr.n
    gen = fused_step.gen_loss(layout, op.n_terms, op.n_terms + op.n_scal, S, spec=spec, d_in=cfg["d_in"])
    out = {}
    for lo in (0, 1):
        lds = lib.tdq_jet_fused_lds(cfg["d_in"], jet_hip._warg(cfg), cfg["d_out"], cfg["n_hidden"], S, lo)
        out["bf16x3" if lo else "bf16"] = fused_step.kernel_source(S, nso, cfg["n_hidden"] - 1, lds, gen, lo=bool(lo))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="/tmp/fused_step_src")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    for name, src in sources().items():
        path = os.path.join(a.out, f"fused_step_{name}.hip")
        with open(path, "w") as f:
            f.write(src.replace('extern "C" __global__', '#include <hip/hip_runtime.h>\nextern "C" __global__', 1))
        r = subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fno-slp-vectorize",
                            "-munsafe-fp-atomics", "--cuda-device-only", "-c", path, "-o", path + ".o",
                            "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
        print(f"== {name} (rc {r.returncode})")
        for ln in r.stderr.splitlines():
            if "remark" in ln or "error" in ln:
                print("  " + ln.split("remark: ")[-1])


if __name__ == "__main__":
    main()
