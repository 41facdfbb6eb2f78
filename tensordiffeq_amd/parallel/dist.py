"""Data parallelism over collocation-point shards: one process per GPU, RCCL over xGMI.

Reference: ``tf.distribute.MirroredStrategy`` in one process (models.py:230-277, fit.py:150-224),
gradients all-reduced with NcclAllReduce inside ``apply_gradients`` (fit.py:180) - but each
replica recomputed the *full* loss (B3), so there was no speed-up.

Design here:
* ``torch.distributed`` with backend ``"nccl"`` (= RCCL on ROCm) on GPUs, ``"gloo"`` on CPU;
  rendezvous from the usual ``RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR`` env variables.
* Collocation points **and their self-adaptive weights** are block-sharded by rank; residual
  means use the *global* point count as denominator, boundary terms are computed on every rank
  and scaled by ``1/world`` - so the SUM over ranks of per-rank losses/grads is exactly the
  single-device full-batch loss/grad.
* One contiguous fp32 bucket per step ``[grad theta | grad(BC lambdas) | loss terms]`` is
  all-reduced (SUM).  For the 50k-parameter Allen-Cahn net that is ~196 KiB: a latency-bound
  message, so a single collective per step is the right shape for xGMI's point-to-point links.
* Parameters are broadcast from rank 0 at start, so every rank starts from identical weights.
* Forced DP (``TDQ_FORCE_DP=1`` or ``init_distributed(force=True)``): a real process group even at
  world 1, so the DP machinery - split or single HIP graph around the collective, bucket packing,
  RCCL itself - runs (and is tested / timed) on a one-GPU box; at world 1 it must reproduce the
  single-process trajectory.
* ``graph_collectives``: with RCCL (or the peer all-reduce) the bucket all-reduce is captured
  INSIDE the step's HIP graph (one replay per step, no host-launched collective); plain gloo, or
  ``TDQ_DP_GRAPH=0``, keeps the two-graph split with the collective launched from the host.
* Peer all-reduce (``parallel/peer.py``, ``csrc/peer.hip``): GPU ranks on one host may replace
  ``dist.all_reduce`` of the fp32 bucket with a one-shot push over xGMI (self-tested and, in
  ``auto`` mode, timed against RCCL at start-up; ``ctx.allreduce_info`` records the choice).
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist


class DistContext:
    def __init__(self, rank=0, world=1, local_rank=0, device=None, backend=None, initialized=False,
                 forced=False):
        self.rank = rank
        self.world = world
        self.local_rank = local_rank
        self.device = device if device is not None else torch.device("cpu")
        self.backend = backend
        self.initialized = initialized
        self.forced = forced
        self.peer = None            # parallel.peer.PeerComm when the one-shot all-reduce is on
        self.retired_peers = []     # communicators settle() switched away from (kept allocated)
        self.allreduce_info = {"impl": "torch.distributed"}

    @property
    def is_distributed(self):
        return self.initialized and (self.world > 1 or self.forced)

    @property
    def graph_collectives(self):
        """Capture the per-step all-reduce inside the step's HIP graph (RCCL only)."""
        return (self.is_distributed and (self.backend == "nccl" or self.peer is not None)
                and self.device.type == "cuda" and os.environ.get("TDQ_DP_GRAPH", "1") != "0")

    def capturable(self, n_floats):
        """Whether an all-reduce of ``n_floats`` fp32 may be captured in a HIP graph: RCCL always;
        under another backend (the gloo rehearsal) only when the peer kernel takes the buffer -
        a larger one would fall back to a host collective, which cannot run inside a capture."""
        if not self.graph_collectives:
            return False
        if self.backend == "nccl":
            return True
        return self.peer is not None and int(n_floats) <= self.peer.cap

    def barrier(self):
        if self.is_distributed:
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()

    def all_reduce_(self, buf):
        if self.is_distributed:
            if self.peer is not None and self.peer.accepts(buf):
                self.peer.all_reduce_(buf)
            else:
                dist.all_reduce(buf, op=dist.ReduceOp.SUM)
        return buf

    def settle_collective(self, n_floats):
        """Collective: re-decide peer vs RCCL at the step's real bucket size (parallel/peer.py
        ``settle``, in-graph replay timings); no-op without a peer communicator."""
        if self.is_distributed and self.peer is not None:
            from . import peer
            peer.settle(self, n_floats)

    def check_health(self):
        """Raise if the peer all-reduce ever timed out waiting for a rank (read at the
        progress / NaN-check cadence, never inside a step)."""
        for comm in ([self.peer] if self.peer is not None else []) + self.retired_peers:
            comm.check()

    def broadcast_(self, buf, src=0):
        if self.is_distributed:
            dist.broadcast(buf, src=src)
        return buf

    def max_scalar(self, v):
        if not self.is_distributed:
            return float(v)
        t = torch.tensor([float(v)], dtype=torch.float64, device=self.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def min_scalar(self, v):
        return -self.max_scalar(-float(v))

    def __repr__(self):
        return (f"DistContext(rank={self.rank}, world={self.world}, device={self.device}, "
                f"backend={self.backend})")


_CTX = None


def env_world():
    return int(os.environ.get("WORLD_SIZE", "1"))


def force_dp_requested():
    return os.environ.get("TDQ_FORCE_DP", "0") == "1"


def free_port(lo=20000, hi=32000):
    """A bindable 127.0.0.1 port for a rendezvous, drawn from [lo, hi) - below Linux's ephemeral
    range (32768+), so the other ranks' outgoing connections cannot be handed the same port before
    rank 0's store binds it (a port from bind(0) is an ephemeral one: EADDRINUSE races)."""
    import random
    import socket
    rng = random.Random()
    for _ in range(200):
        port = rng.randrange(lo, hi)
        with socket.socket() as s:
            try:
                s.bind(("127.0.0.1", port))
            except OSError:
                continue
        return port
    raise RuntimeError(f"no free port in [{lo}, {hi})")


_free_port = free_port


# rank variables of launchers that start one process per task themselves (torchrun, Slurm srun,
# Open MPI / MPICH / MVAPICH mpirun, PMIx): such a process must never self-launch more ranks
_LAUNCHER_VARS = ("WORLD_SIZE", "SLURM_PROCID", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE", "PMIX_RANK",
                  "MV2_COMM_WORLD_SIZE")


def launcher_env():
    """True when a launcher (torchrun / torch.distributed.run / srun / an MPI-style wrapper)
    already set up this process as one rank."""
    return any(v in os.environ for v in _LAUNCHER_VARS)


def _interactive_shell():
    """True inside a Jupyter kernel (``ipykernel`` is the kernel process itself) or a running
    IPython shell.  A library that merely imports IPython does not make a plain script interactive,
    so for IPython the test is whether an IPython instance exists, not whether the module is loaded."""
    import sys
    if "ipykernel" in sys.modules:
        return True
    ip = sys.modules.get("IPython")
    if ip is None:
        return False
    try:
        return ip.get_ipython() is not None
    except Exception:  # noqa: BLE001 - a broken / partial IPython import: not a shell
        return False


def relaunch_argv():
    """The arguments that re-run this program under ``torch.distributed.run``, or None when it
    is not a plain script / module run (an interactive interpreter, a Jupyter / IPython kernel,
    ``python -c``, an embedding host): those must train at world 1 rather than re-run
    something else N times.  ``python -m pkg.mod args`` -> ``-m pkg.mod args``."""
    import sys
    if hasattr(sys, "ps1") or _interactive_shell():
        return None
    main = sys.modules.get("__main__")
    argv = list(sys.argv)
    if main is None or not argv or not argv[0] or argv[0] == "-c":
        return None
    spec = getattr(main, "__spec__", None)
    if spec is not None and getattr(spec, "name", None) and spec.name != "__main__":
        mod = spec.name[:-len(".__main__")] if spec.name.endswith(".__main__") else spec.name
        return ["-m", mod] + argv[1:]
    f = getattr(main, "__file__", None)
    if not f or not os.path.exists(argv[0]) or os.path.abspath(f) != os.path.abspath(argv[0]):
        return None
    return argv


def visible_devices():
    """Number of GPUs this process could use.  ``torch.cuda.device_count()`` does not
    initialise the HIP runtime, so this is safe before a self-launch (``TDQ_DIST_NPROC``
    overrides: tests rehearse the self-launch on CPU ranks)."""
    env = os.environ.get("TDQ_DIST_NPROC")
    if env:
        return int(env)
    return torch.cuda.device_count()


def self_launch(nproc, argv=None, env=None):
    """Run the current program as ``nproc`` ranks of one node and return their exit code.

    The reference's ``compile(..., dist=True)`` uses every visible GPU from a plain ``python``
    process (``tf.distribute.MirroredStrategy``, tensordiffeq/models.py:230-243).  Here DP is
    one process per GPU, so a plain process that asks for DP re-runs its own script under
    ``torch.distributed.run`` as CHILD processes (never ``exec``: this process may already hold
    the GPU), streams their output through and exits with their code.  Rendezvous on
    127.0.0.1 with a free port."""
    import subprocess
    import sys
    argv = relaunch_argv() if argv is None else list(argv)
    if not argv or not argv[0] or argv[0] == "-c" or (argv[0] != "-m" and not os.path.exists(argv[0])):
        raise RuntimeError("cannot self-launch ranks: the program was not started from a script file; "
                           "use 'python -m torch.distributed.run --nproc-per-node N script.py'")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={int(nproc)}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + argv
    child_env = dict(os.environ if env is None else env)
    child_env["TDQ_SELF_LAUNCHED"] = "1"
    child_env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    child_env.pop("TDQ_DIST_NPROC", None)
    r = subprocess.run(cmd, env=child_env)
    return r.returncode


def maybe_self_launch(n=None, why="dist=True"):
    """Relaunch as ``n`` ranks (default: every visible device) when no launcher set this process
    up and more than one device is visible; returns normally only when this process should go
    on at world 1 (it prints why).  ``TDQ_DIST_AUTOLAUNCH=0`` disables the relaunch."""
    import sys
    import warnings
    if launcher_env() or os.environ.get("TDQ_SELF_LAUNCHED") == "1":
        return
    n = visible_devices() if n is None else int(n)
    if n > 1 and "PYTEST_CURRENT_TEST" in os.environ:
        # never re-run a test runner as N ranks
        warnings.warn(f"{why}: {n} devices visible but running under pytest - training at world 1", stacklevel=3)
        return
    if n <= 1:
        warnings.warn(f"{why}: one visible device and no launcher - training at world 1 "
                      "(launch with 'torch.distributed.run --nproc-per-node N' for N ranks)", stacklevel=3)
        return
    if os.environ.get("TDQ_DIST_AUTOLAUNCH", "1") == "0":
        warnings.warn(f"{why}: {n} devices visible but TDQ_DIST_AUTOLAUNCH=0 and no launcher - training at "
                      "world 1", stacklevel=3)
        return
    if relaunch_argv() is None:
        warnings.warn(f"{why}: {n} devices visible but this is not a plain script or module run (interactive "
                      "session, notebook kernel, python -c) - training at world 1; launch with "
                      "'torch.distributed.run --nproc-per-node N' for N ranks", stacklevel=3)
        return
    print(f"[tensordiffeq_amd] {why}: launching {n} ranks (one per device) with torch.distributed.run",
          file=sys.stderr, flush=True)
    sys.stdout.flush()
    rc = self_launch(n)
    sys.exit(rc)


def init_distributed(backend=None, device=None, timeout_s=600, force=None, auto_launch=False):
    """Initialise (once) from the torchrun environment; returns the process' DistContext.
    ``force`` (default ``TDQ_FORCE_DP``): build the process group even at world 1.
    ``auto_launch``: with no launcher and several visible devices, re-run this program as one
    rank per device first (:func:`maybe_self_launch`; the solver's ``compile(dist=True)``)."""
    global _CTX
    if _CTX is not None:
        return _CTX
    force = force_dp_requested() if force is None else bool(force)
    if auto_launch and not force:
        maybe_self_launch()
    world = env_world()
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    if device is None:
        if torch.cuda.is_available():
            device = torch.device("cuda", local_rank % max(1, torch.cuda.device_count()))
        else:
            device = torch.device("cpu")
    device = torch.device(device)
    if device.type == "cuda":
        torch.cuda.set_device(device)
    if backend is None:
        # TDQ_DIST_BACKEND=gloo: rehearse the multi-rank GPU path with several ranks sharing one GPU
        # (RCCL refuses two ranks on one device); the peer all-reduce then carries the bucket
        backend = os.environ.get("TDQ_DIST_BACKEND") or ("nccl" if device.type == "cuda" else "gloo")
    initialized = False
    if world > 1 or force:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500" if world > 1 else str(_free_port()))
        if not dist.is_initialized():
            kw = {}
            if backend == "nccl":
                kw["device_id"] = device
            dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                    timeout=datetime.timedelta(seconds=timeout_s), **kw)
        initialized = True
    _CTX = DistContext(rank, world, local_rank, device, backend, initialized, forced=force and world == 1)
    if initialized and world > 1 and device.type == "cuda":
        from . import peer
        _CTX.peer = peer.setup(_CTX)
    return _CTX


def get_context(device=None):
    """Current context; a trivial single-process one when never initialised."""
    if _CTX is not None:
        return _CTX
    if device is None:
        device = torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")
    return DistContext(0, 1, 0, torch.device(device), None, False)


def reset_context():
    global _CTX
    _CTX = None


def shard_range(n, rank, world):
    """Balanced contiguous block ``[lo, hi)`` of ``n`` items for ``rank``."""
    base, rem = divmod(n, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def shard(t, rank, world):
    lo, hi = shard_range(t.shape[0], rank, world)
    return t[lo:hi]


def destroy():
    global _CTX
    if _CTX is not None:
        for comm in ([_CTX.peer] if _CTX.peer is not None else []) + _CTX.retired_peers:
            comm.close()
        _CTX.peer = None
        _CTX.retired_peers = []
    if dist.is_initialized():
        dist.destroy_process_group()
    _CTX = None
