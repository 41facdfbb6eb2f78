"""Wall-clock split of the AC-SA Adam phase on one GPU: problem build, program build (trace +
plan + fused loss), first fit step (graph capture), steady-state steps.  One JSON line."""
import json
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "examples"))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    import importlib.util
    spec = importlib.util.spec_from_file_location("ac_sa", os.path.join(os.path.dirname(HERE), "examples", "AC-SA.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    args = mod.parser("x", iters=10, newton=0).parse_args(["--precision", "bf16", "--quiet"])
    sync = torch.cuda.synchronize
    t0 = time.perf_counter()
    model, _ = mod.build(args)
    sync()
    t1 = time.perf_counter()
    model.program()
    sync()
    t2 = time.perf_counter()
    model.fit(tf_iter=1)
    sync()
    t3 = time.perf_counter()
    model.fit(tf_iter=1000)
    sync()
    t4 = time.perf_counter()
    model.fit(tf_iter=1000)
    sync()
    t5 = time.perf_counter()
    print(json.dumps({"build_s": t1 - t0, "program_s": t2 - t1, "first_fit_1step_s": t3 - t2,
                      "fit_1000_first_s": t4 - t3, "fit_1000_again_s": t5 - t4}), flush=True)


if __name__ == "__main__":
    main()
