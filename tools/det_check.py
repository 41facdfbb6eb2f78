"""Determinism probe of the one-launch fused objective: ``[grad | loss]`` evaluated repeatedly in
one process (bitwise), and its sha printed so two processes can be compared."""
import hashlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from tensordiffeq_amd.fit import LossGradEngine
    for prec in sys.argv[1:] or ("bf16", "bf16x3"):
        m = bench.build_problem(4096, 1, "hip", torch.device("cuda", 0), False, prec)
        eng = LossGradEngine(m, m.program(), m.lambdas)
        hs, firsts, alld = [], set(), set()
        ref = None
        for _ in range(51):
            fg = eng.evaluate_fg().clone()
            if ref is None:
                ref = fg
            elif not torch.equal(fg, ref):
                nz = torch.nonzero(fg != ref)[:, 0].tolist()
                firsts.add(int(nz[0]))
                alld.update(nz)
            hs.append(hashlib.sha256(fg.cpu().numpy().tobytes()).hexdigest()[:12])
        torch.cuda.synchronize()
        print(f"{prec} [{os.environ.get('TDQ_FUSED_STEP_DEFINES', '')}]: first sha {hs[0]}, {len(set(hs))} distinct results in 51 evaluations "
              f"(first differing indices {sorted(firsts)[:6]}); {len(alld)} entries ever differ: {sorted(alld)[:24]}")


if __name__ == "__main__":
    main()
