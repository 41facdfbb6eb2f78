"""Point ranges for concurrent graph branches (fit.point_ranges) and the fused loss's block
alignment that makes them possible (ops/loss_fused.py: LFGroup.phase).  CPU: geometry only; the
GPU equivalence (bitwise equal trajectories) is tests/test_hip_kernels.py::
test_point_ranges_match_single_launch."""
import math

import numpy as np
import pytest
import torch

import tensordiffeq_amd as tdq
from tensordiffeq_amd import fit, fusion
from tensordiffeq_amd.boundaries import IC, DomainND, periodicBC
from tensordiffeq_amd.ops.loss_fused import LF_BLOCK, FusedLossOp


def _program(n_f=20000):
    tdq.set_seed(0)
    D = DomainND(["x", "t"], time_var="t")
    D.add("x", [-1.0, 1.0], 512)
    D.add("t", [0.0, 1.0], 201)
    D.generate_collocation_points(n_f)

    def deriv_model(u_model, x, t):
        u = u_model(torch.cat([x, t], 1))
        return u, tdq.grad(u, x)

    def f_model(u_model, x, t):
        u = u_model(torch.cat([x, t], 1))
        return tdq.grad(u, t) - 1e-4 * tdq.grad(tdq.grad(u, x), x) + 5.0 * u ** 3 - 5.0 * u

    m = tdq.CollocationSolverND(verbose=False)
    m.compile([2, 128, 128, 128, 128, 1], f_model, D,
              [IC(D, [lambda x: x ** 2 * np.cos(math.pi * x)], var=[["x"]]), periodicBC(D, ["x"], [deriv_model])],
              Adaptive_type="self-adaptive", dict_adaptive={"residual": [True], "BCs": [True, False]},
              init_weights={"residual": [torch.rand(n_f, 1)], "BCs": [100 * torch.rand(512, 1), None]},
              backend="jet", device="cpu")
    prog = m.program()
    fl = fusion.build(prog, m.lambdas)
    return prog, FusedLossOp(fl, prog, m.lambdas, [], fl.lam_offsets)


def test_single_segment_blocks_start_on_multiples_of_128():
    prog, fop = _program()
    res = [s for s in prog.segments if s.name == "residual"][0]
    assert res.offset % LF_BLOCK != 0                     # BC segments come first (914 points)
    spans = [sp for sp in fop.block_spans if sp[0] >= res.offset]
    assert spans[0][0] == res.offset and spans[0][1] == (res.offset // LF_BLOCK + 1) * LF_BLOCK - 1
    assert all(lo % LF_BLOCK == 0 for lo, _ in spans[1:])
    assert spans[-1][1] == res.offset + res.n - 1
    covered = sum(hi - lo + 1 for lo, hi in spans)
    assert covered == res.n


def test_split_block_cuts_cleanly():
    prog, fop = _program()
    for a in (2048, 8320, 15360):
        b = fop.split_block(a)
        assert b is not None
        assert all(hi < a for _, hi in fop.block_spans[:b])
        assert all(lo >= a for lo, _ in fop.block_spans[b:])
    assert fop.split_block(1) is None                     # inside the first IC block


@pytest.mark.parametrize("spec,n", [("auto", 2), ("0.3", 2), ("0", 0), ("off", 0)])
def test_point_ranges_partition(spec, n, monkeypatch):
    prog, fop = _program()
    monkeypatch.setenv("TDQ_SPLIT", spec)
    prog.precision = "bf16"
    r = fit.point_ranges(prog, fop)
    if n == 0:
        assert r is None
        return
    assert len(r) == n
    N = prog.X_all.shape[0]
    assert r[0][0] == 0 and r[-1][1] == N and r[0][2] == 0 and r[-1][2] + r[-1][3] == fop.n_blocks
    for (lo, hi, b0, nb), nxt in zip(r, r[1:] + [None]):
        assert lo % 128 == 0 and (hi == N or hi % 128 == 0)
        if nxt is not None:
            assert nxt[0] == hi and nxt[2] == b0 + nb


def test_point_ranges_skip_small_problems(monkeypatch):
    prog, fop = _program(n_f=3000)
    prog.precision = "bf16"
    monkeypatch.setenv("TDQ_SPLIT", "auto")
    assert fit.point_ranges(prog, fop) is None


def test_point_ranges_one_cut_at_most(monkeypatch):
    prog, fop = _program()
    prog.precision = "bf16"
    monkeypatch.setenv("TDQ_SPLIT", "0.3,0.6")
    with pytest.raises(ValueError):
        fit.point_ranges(prog, fop)


def test_cut_on_slab_chunk_boundary_enables_prereduce(monkeypatch):
    """bf16 (128-point backward workgroups): the auto cut lands on a row boundary of the slab
    reduction's chunks, so the first range's chunks are pre-reduced (fit.prereduce_chunk); a cut
    off the boundaries disables it.  Needs the native library only for the geometry query."""
    from tensordiffeq_amd.ops import _lib, jet_hip
    from tensordiffeq_amd.ops.jet_mlp import hip_config
    if not _lib.available():
        pytest.skip("native library not built")
    prog, fop = _program(n_f=50000)
    prog.precision = "bf16"
    monkeypatch.setenv("TDQ_SPLIT", "auto")
    r = fit.point_ranges(prog, fop)
    N = prog.X_all.shape[0]
    pts_b, nwg, chunks, _ = jet_hip.slab_geometry(hip_config(prog.net, prog.plan, "bf16"), N)
    assert pts_b == 128 and nwg == (N + 127) // 128 and chunks == 8
    c = fit.prereduce_chunk(prog, r)
    assert 0 < c < chunks and r[0][1] == (nwg * c // chunks) * pts_b
    assert abs(r[0][1] - 0.38 * N) <= 0.05 * N
    monkeypatch.setenv("TDQ_PREREDUCE", "0")
    assert fit.prereduce_chunk(prog, r) == 0
    monkeypatch.delenv("TDQ_PREREDUCE")
    off = [(0, r[0][1] + 128) + r[0][2:], (r[0][1] + 128,) + r[1][1:]]
    assert fit.prereduce_chunk(prog, off) == 0
