"""Recompute backward (csrc/jet_bwdr.h): the forward writes only the jets, the backward re-runs the
forward on chip (activations in registers / one layer through the saved buffer) - gradients,
losses and a short fused-tail trajectory must match the saved-activation kernel pair (same MFMA
sequence, same bits for the activations; only the slab partition, 64 vs 128 points per row,
changes the summation order)."""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(on, n_f=5000, steps=16):
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import bench
    from tensordiffeq_amd.ops import jet_hip
    from tensordiffeq_amd.ops.jet_mlp import hip_config
    jet_hip.set_bwd_recompute(on)
    try:
        m = bench.build_problem(n_f, 1, "hip", torch.device("cuda", 0), False, "bf16")
        prog = m.program()
        active = jet_hip.bwd_recompute_active(hip_config(prog.net, prog.plan, prog.precision))
        loss, grads = m.grad()
        g = [x.detach().clone() for x in grads]
        loss = float(loss)
        m.fit(tf_iter=steps)
        hist = [h["Total Loss"] for h in m.losses]
        return active, loss, g, hist, m.u_model.flat.detach().clone()
    finally:
        jet_hip.set_bwd_recompute(False)


@pytest.mark.timeout(300)
def test_bwdr_matches_saved_activation_backward():
    a_on, l_on, g_on, h_on, f_on = _run(True)
    a_off, l_off, g_off, h_off, f_off = _run(False)
    assert a_on and not a_off
    print(f"BWDR loss {l_on:.7e} vs {l_off:.7e}")
    assert abs(l_on - l_off) <= 1e-6 * abs(l_off)
    for x, y in zip(g_on, g_off):
        err = ((x - y).norm() / y.norm().clamp_min(1e-30)).item()
        print(f"BWDR grad rel err {err:.3e}")
        assert err < 2e-3
    print("BWDR hist", h_on[-1], h_off[-1])
    assert h_on == pytest.approx(h_off, rel=2e-3)
    assert ((f_on - f_off).norm() / f_off.norm()).item() < 2e-3
