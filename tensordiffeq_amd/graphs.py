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
    """
    was_enabled = gc.isenabled()
    gc.disable()
    try:
        with torch.cuda.graph(graph, pool=pool):
            yield
    finally:
        if was_enabled:
            gc.enable()
