"""HIP-graph capture helper shared by the training engines (fit.py) and the device L-BFGS."""
from __future__ import annotations

import contextlib
import gc

import torch


@contextlib.contextmanager
def capture_graph(graph, pool=None):
    """``torch.cuda.graph`` with the Python garbage collector paused for the capture.

    ``torch.cuda.graph`` collects once before capturing, but a collection triggered by an
    allocation INSIDE the capture can run destructors that make HIP calls a capturing stream
    forbids (event / graph-exec / stream release) and invalidate the capture or abort the process.

    With a process group up, the capture is thread-local: the RCCL watchdog thread keeps querying
    the completion events of earlier collectives, which a global-mode capture turns into
    ``hipErrorStreamCaptureUnsupported`` and a process abort (seen on MI355X with the all-reduce
    captured in the DP step graph).
    """
    was_enabled = gc.isenabled()
    gc.disable()
    import torch.distributed as dist
    mode = "thread_local" if (dist.is_available() and dist.is_initialized()) else "global"
    try:
        with torch.cuda.graph(graph, pool=pool, capture_error_mode=mode):
            yield
    finally:
        if was_enabled:
            gc.enable()
