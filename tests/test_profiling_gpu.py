"""Built-in profiler on the GPU: graph-replayed HIP kernels appear in the kernel table."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_profile_sees_graph_replayed_jet_kernels(tmp_path, monkeypatch):
    import bench
    from tensordiffeq_amd import profiling
    monkeypatch.setenv("TDQ_PROFILE", str(tmp_path / "p"))
    monkeypatch.setattr(profiling, "_FIT_CALLS", [0])
    m = bench.build_problem(2048, 1, "hip", torch.device("cuda", 0), False)
    m.fit(tf_iter=5)
    text = (tmp_path / "p" / "fit_0" / "kernels.txt").read_text()
    assert text.splitlines()[1].startswith("# device kernels")
    # the step's point kernel: the one-launch fused step (hipRTC code object; bf16x3 on this
    # solver's default precision) or, outside its envelope, the separate backward
    assert ("tdq_fused_step" in text or "jet_bwd_bf3_kernel" in text), text[:2000]
    assert "adam_multi_kernel" in text or "tail_adam_kernel" in text
    assert os.path.getsize(tmp_path / "p" / "fit_0" / "trace.json") > 0
