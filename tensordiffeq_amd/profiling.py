"""Built-in kernel profiling (SURVEY.md §5 "Tracing / profiling").

The reference only has commented-out ``tf.profiler.experimental.start/stop`` around its loops
(tensordiffeq/fit.py:39,57,59,91,217,219,224).  Here any training call can be wrapped::

    with tdq.profiling.kernel_profile("prof_dir"):
        model.fit(tf_iter=200)

or, without code changes, ``TDQ_PROFILE=prof_dir python script.py`` (every ``fit`` of a solver is
wrapped; call k of the process writes ``prof_dir/fit_<k>/``, so a script that fits several times
- transfer learning, Adam then a separate L-BFGS fit - keeps every call).  The context runs
``torch.profiler`` (CPU + HIP activities) and writes

* ``prof_dir/trace.json``  - Chrome / Perfetto trace of host ops and device kernels,
* ``prof_dir/kernels.txt`` - one row per kernel name: total us, calls, us per call, share
  (the format of the ``profiles/*kernel_stats.txt`` tables that rocprofv3 runs produce).

For PMC counters (MFMA / LDS / HBM) use rocprofv3 (``tools/gpu_runs/r2_pmc.sh``); this is the
in-process view.  Under data parallelism each rank writes ``prof_dir/rank<k>/``.
"""
from __future__ import annotations

import contextlib
import os

import torch


def _device_rows(prof):
    """(name, total us, calls) of device kernels only (operator events would double count)."""
    from torch.autograd import DeviceType
    agg = {}
    for ev in prof.events():
        if ev.device_type != DeviceType.CUDA:
            continue
        us = ev.time_range.elapsed_us()
        tot, n = agg.get(ev.name, (0.0, 0))
        agg[ev.name] = (tot + us, n + 1)
    return sorted(((k, t, n) for k, (t, n) in agg.items()), key=lambda r: -r[1])


def _host_rows(prof):
    """(name, self CPU us, calls) of host ops (CPU-only runs)."""
    rows = [(ev.key, ev.self_cpu_time_total, ev.count) for ev in prof.key_averages()
            if ev.self_cpu_time_total > 0]
    return sorted(rows, key=lambda r: -r[1])


def write_kernel_table(prof, path, title=""):
    """Kernel table from a finished ``torch.profiler.profile``: device kernels when any were
    recorded, host ops (self time) otherwise (CPU-only runs)."""
    rows, kind = _device_rows(prof), "device kernels"
    if not rows:
        rows, kind = _host_rows(prof), "host ops (self time)"
    total = sum(r[1] for r in rows) or 1.0
    with open(path, "w") as f:
        if title:
            f.write(f"# {title}\n")
        f.write(f"# {kind}: total_us  calls  us_per_call  pct  name\n")
        for name, us, n in rows:
            f.write(f"{us:12.1f} {n:6d} {us / max(1, n):10.2f} {100 * us / total:5.1f}%  {name[:150]}\n")
    return rows


@contextlib.contextmanager
def kernel_profile(out_dir, rank=None, title=""):
    """Profile the enclosed block; see the module docstring for the outputs."""
    if rank is None:
        rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    d = os.path.join(out_dir, f"rank{rank}") if world > 1 else out_dir
    os.makedirs(d, exist_ok=True)
    acts = [torch.profiler.ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(torch.profiler.ProfilerActivity.CUDA)
    with torch.profiler.profile(activities=acts, record_shapes=False) as prof:
        yield prof
        if torch.cuda.is_available():
            torch.cuda.synchronize()
    prof.export_chrome_trace(os.path.join(d, "trace.json"))
    write_kernel_table(prof, os.path.join(d, "kernels.txt"), title=title)


_FIT_CALLS = [0]


def env_profile_dir():
    """``TDQ_PROFILE`` (a directory) or None."""
    return os.environ.get("TDQ_PROFILE") or None


@contextlib.contextmanager
def maybe_profile(title=""):
    """``kernel_profile`` when ``TDQ_PROFILE`` is set, else a no-op."""
    d = env_profile_dir()
    if d is None:
        yield None
        return
    k = _FIT_CALLS[0]
    _FIT_CALLS[0] += 1
    with kernel_profile(os.path.join(d, f"fit_{k}"), title=title) as prof:
        yield prof
