"""Train the flagship AC-SA problem with the reference schedule and report the L2 error.

Runs examples/AC-SA.py (Adam ``--iters`` + L-BFGS ``--newton``) for each requested precision and
prints one JSON line per run: relative L2 on the AC.mat grid, final/min losses, wall time per
phase.  Usage (GPU):  python tools/accuracy_ac_sa.py --iters 10000 --newton 10000 --prec bf16x3 fp32 bf16+bf16x3
(``a+b``: Adam phase in precision a, L-BFGS phase in b).
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "examples"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10000)
    ap.add_argument("--newton", type=int, default=10000)
    ap.add_argument("--prec", nargs="+", default=["bf16x3"])
    ap.add_argument("--seed", type=int, default=0)
    args = ap.parse_args()
    import importlib.util
    spec = importlib.util.spec_from_file_location("ac_sa", os.path.join(os.path.dirname(HERE), "examples", "AC-SA.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    for p in args.prec:  # "adam+lbfgs" (e.g. bf16+bf16x3) picks a per-phase precision
        pa, _, pn = p.partition("+")
        extra = ["--newton-precision", pn] if pn else []
        res = mod.main(["--iters", str(args.iters), "--newton", str(args.newton), "--precision", pa,
                        "--seed", str(args.seed), "--quiet"] + extra)
        res["precision"] = p
        res["schedule"] = f"adam {args.iters} + lbfgs {args.newton}"
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
