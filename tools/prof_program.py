"""cProfile of CollocationSolverND.program() (trace + plan + fused-loss build) for the AC-SA example
(run from the repo root on the GPU box): python tools/prof_program.py"""
import cProfile, pstats, os, sys, io, importlib.util
sys.path.insert(0, "examples"); sys.path.insert(0, ".")
spec = importlib.util.spec_from_file_location("ac_sa", "examples/AC-SA.py")
mod = importlib.util.module_from_spec(spec); spec.loader.exec_module(mod)
args = mod.parser("x", iters=10, newton=0).parse_args(["--precision", "bf16", "--quiet"])
model, _ = mod.build(args)
import torch; torch.cuda.synchronize()
pr = cProfile.Profile(); pr.enable(); model.program(); torch.cuda.synchronize(); pr.disable()
s = io.StringIO(); pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(45); print(s.getvalue())
