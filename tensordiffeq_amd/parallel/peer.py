"""One-shot peer-memory all-reduce over xGMI (``csrc/peer.hip``) for the per-step DP bucket.

The reference all-reduces gradients with NCCL inside ``MirroredStrategy.apply_gradients``
(``tensordiffeq/fit.py:150-224``).  Here the message is one ~196 KiB fp32 bucket per ~0.2 ms step:
latency, not bandwidth, decides.  RCCL's ring pays 2 (world - 1) hops; MI355X nodes wire every GPU
pair with its own xGMI link, so :class:`PeerComm` lets each rank write its bucket straight into a
receive slot of every peer (one hop, all links at once) and sum the world copies in rank order
(bitwise identical on every rank).  The receive slots and flags live in one uncached device
allocation per rank, shared with ``hipIpcGetMemHandle`` / ``hipIpcOpenMemHandle``; the handle
exchange rides on the torch.distributed process group (RCCL or gloo).

:func:`setup` runs collectively from :func:`..parallel.dist.init_distributed` on GPU ranks of one
host: it builds the communicator, self-tests it (three calls, both receive parities, exact integer
data checked on every rank) and - in ``auto`` mode - times it against ``dist.all_reduce`` on a
bucket-sized buffer, keeping whichever is faster (decided on the max over ranks, so every rank
agrees).  Any failure on any rank disables it on all ranks (``dist.all_reduce`` stays).
``TDQ_PEER_ALLREDUCE``: ``auto`` (default), ``1`` (use it whenever the self-test passes), ``0``.
"""
from __future__ import annotations

import ctypes
import os
import socket
import time

import torch
import torch.distributed as dist

from ..ops import _lib

_KINDS = {0: "uncached", 1: "fine-grained", 2: "coarse"}


def mode():
    m = os.environ.get("TDQ_PEER_ALLREDUCE", "auto").strip().lower()
    return m if m in ("auto", "0", "1") else "auto"


class PeerComm:
    """Peer receive slots + flags of every rank mapped into this process; :meth:`all_reduce_` sums
    a contiguous fp32 CUDA tensor over ranks in place (one kernel on the current stream).

    Construct on every rank at the same time (the IPC handles are all-gathered)."""

    def __init__(self, rank, world, device, cap_floats=None, kind=None, timeout_s=None):
        lib = _lib.load(required=True)
        self.lib, self.rank, self.world, self.device = lib, rank, world, torch.device(device)
        self.maxw, self.chunk = lib.tdq_peer_maxw(), lib.tdq_peer_chunk()
        if not 1 <= world <= self.maxw:
            raise ValueError(f"peer all-reduce supports 1..{self.maxw} ranks, got {world}")
        cap = int(cap_floats or os.environ.get("TDQ_PEER_CAP", 1 << 20))
        self.cap = (cap + self.chunk - 1) // self.chunk * self.chunk
        self.max_blocks = self.cap // self.chunk
        self.recv_bytes = 2 * self.maxw * self.cap * 4
        flag_bytes = self.maxw * self.max_blocks * 4
        self.timeout_ticks = int(float(timeout_s or os.environ.get("TDQ_PEER_TIMEOUT_S", 30)) * 1e8)
        self._base = ctypes.c_void_p(0)
        self._opened = []
        kinds = [kind] if kind is not None else [0, 1, 2]
        rc = -1
        for k in kinds:
            rc = lib.tdq_peer_alloc(self.recv_bytes + flag_bytes, k, ctypes.byref(self._base))
            if rc == 0:
                self.kind = k
                break
        _lib.check(rc, "tdq_peer_alloc")
        self.seqs = torch.zeros(self.max_blocks, dtype=torch.int32, device=self.device)
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        self._recv = (ctypes.c_void_p * world)()
        self._flag = (ctypes.c_void_p * world)()

    # -- collective setup ------------------------------------------------------------------
    def handle(self):
        h = ctypes.create_string_buffer(64)
        _lib.check(self.lib.tdq_peer_ipc_handle(self._base, h), "hipIpcGetMemHandle")
        return bytes(h.raw)

    def open_peers(self, handles):
        """Map every peer's region (``handles[q]``: rank q's 64-byte IPC handle)."""
        for q in range(self.world):
            if q == self.rank:
                base = self._base.value
            else:
                p = ctypes.c_void_p(0)
                _lib.check(self.lib.tdq_peer_ipc_open(ctypes.create_string_buffer(handles[q], 64), ctypes.byref(p)),
                           f"hipIpcOpenMemHandle(rank {q})")
                self._opened.append(p)
                base = p.value
            self._recv[q] = base
            self._flag[q] = base + self.recv_bytes

    # -- data path -------------------------------------------------------------------------
    def accepts(self, buf):
        return (buf.is_cuda and buf.dtype == torch.float32 and buf.is_contiguous() and buf.numel() <= self.cap
                and buf.data_ptr() % 16 == 0 and buf.device == self.device)

    def all_reduce_(self, buf):
        rc = self.lib.tdq_peer_allreduce(_lib.ptr(buf), buf.numel(), self.rank, self.world, self.cap,
                                         self.max_blocks, self._recv, self._flag, _lib.ptr(self.seqs),
                                         _lib.ptr(self.err), self.timeout_ticks, _lib.stream_ptr(self.device))
        _lib.check(rc, "tdq_peer_allreduce")
        return buf

    def check(self):
        """Raise if a wait ever timed out (a peer did not arrive within TDQ_PEER_TIMEOUT_S)."""
        if int(self.err.item()) != 0:
            raise RuntimeError(f"peer all-reduce: rank {self.rank} timed out waiting for a peer "
                               f"(TDQ_PEER_TIMEOUT_S); results of the steps since the last check are invalid")

    def close(self):
        torch.cuda.synchronize(self.device)
        for p in self._opened:
            self.lib.tdq_peer_ipc_close(p)
        self._opened = []
        if self._base.value:
            self.lib.tdq_peer_free(self._base)
            self._base = ctypes.c_void_p(0)


def _log(msg):
    if os.environ.get("TDQ_PEER_DEBUG", "0") == "1":
        import sys
        print(f"[peer rank {os.environ.get('RANK', '?')}] {msg}", file=sys.stderr, flush=True)


def _gather(obj, world):
    out = [None] * world
    dist.all_gather_object(out, obj)
    return out


def _self_test(comm, n):
    """Three calls (both receive parities, then the first again) on exact small integers."""
    ok = True
    idx = torch.arange(n, device=comm.device, dtype=torch.float32)
    for it in range(3):
        buf = (idx.remainder(97) + 1.0) * (comm.rank + 1 + it)
        comm.all_reduce_(buf)
        tot = sum(q + 1 + it for q in range(comm.world))
        want = (idx.remainder(97) + 1.0) * tot
        ok = ok and bool(torch.equal(buf, want))
    torch.cuda.synchronize(comm.device)
    return ok and int(comm.err.item()) == 0


def _time_us(fn, buf, ctx, reps=30):
    """Host-launched per-call time (a collective that cannot be captured: gloo)."""
    for _ in range(3):
        fn(buf)
    torch.cuda.synchronize(buf.device)
    ctx.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn(buf)
    torch.cuda.synchronize(buf.device)
    return (time.perf_counter() - t0) / reps * 1e6


def _time_us_graph(fn, buf, ctx, calls=10, reps=20):
    """Per-call time the way the DP step runs the collective: ``calls`` of them captured in one
    HIP graph, the graph replayed ``reps`` times (bench.allreduce_replay_us measures the same)."""
    from ..graphs import capture_graph
    dev = buf.device
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        fn(buf)
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize(dev)
    g = torch.cuda.CUDAGraph()
    with capture_graph(g):
        for _ in range(calls):
            fn(buf)
    g.replay()
    torch.cuda.synchronize(dev)
    ctx.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) / (reps * calls) * 1e6


def _compare(comm, ctx, n_floats):
    """``(peer us, torch.distributed us)`` per call on an ``n_floats`` buffer, max over ranks: both
    in-graph when the backend's collective can be captured (RCCL), else the torch one host-launched."""
    W = ctx.world
    buf = torch.randn(int(n_floats), device=ctx.device)
    t_peer = _time_us_graph(comm.all_reduce_, buf, ctx)

    def ref(b):
        dist.all_reduce(b, op=dist.ReduceOp.SUM)

    t_ref = _time_us_graph(ref, buf, ctx) if ctx.backend == "nccl" else _time_us(ref, buf, ctx)
    ts = _gather([t_peer, t_ref], W)
    return max(x[0] for x in ts), max(x[1] for x in ts)


def settle(ctx, n_floats):
    """Collective (every rank, same point): re-decide peer vs torch.distributed at the step's REAL
    bucket size with in-graph replay timings (``auto`` mode only; once per size).  Keeps the
    faster; records the timings in ``ctx.allreduce_info["settled"]``."""
    comm = ctx.peer
    if comm is None or mode() != "auto" or ctx.backend != "nccl" or int(n_floats) > comm.cap:
        return
    if ctx.allreduce_info.get("settled", {}).get("floats") == int(n_floats):
        return
    t_peer, t_ref = _compare(comm, ctx, n_floats)
    use = _gather(bool(t_peer < t_ref) and comm.err.item() == 0, ctx.world)
    ctx.allreduce_info["settled"] = {"floats": int(n_floats), "peer_us": round(t_peer, 2),
                                     "torch_us": round(t_ref, 2), "choice": "peer" if all(use) else "torch"}
    if not all(use):
        # route NEW collectives to torch.distributed but keep the communicator (its IPC receive
        # slots and flags) allocated: HIP graphs captured before this point - a cached
        # LossGradEngine graph, another AdamEngine's graphs at another bucket size - may still
        # contain the peer kernel, and replaying them after a close would read freed memory
        ctx.retired_peers.append(comm)
        ctx.peer = None
        ctx.allreduce_info["impl"] = "torch.distributed"
        ctx.allreduce_info["peer"] = "off: slower in-graph at the step's bucket size"


def setup(ctx, bench_floats=49_408):
    """Collectively build, self-test and (``auto``) time the peer all-reduce; returns the
    :class:`PeerComm` to use, or ``None``.  Records what happened in ``ctx.allreduce_info``."""
    m = mode()
    info = {"impl": "torch.distributed", "peer_mode": m}
    ctx.allreduce_info = info
    if m == "0" or ctx.device.type != "cuda" or ctx.world < 2 or not _lib.available():
        return None
    W = ctx.world
    _log("setup: gathering hosts")
    hosts = _gather(socket.gethostname(), W)
    if len(set(hosts)) != 1:
        info["peer"] = "off: ranks on more than one host"
        return None
    comm, err = None, None
    try:
        comm = PeerComm(ctx.rank, W, ctx.device)
        h = comm.handle()
    except Exception as e:  # noqa: BLE001 - reported, every rank falls back together
        h, err = None, f"{type(e).__name__}: {e}"
    _log(f"setup: allocated ({err or 'ok'}), gathering handles")
    handles = _gather(h, W)
    if any(x is None for x in handles):
        info["peer"] = f"off: setup failed ({err or 'on another rank'})"
        if comm is not None:
            comm.close()
        return None
    try:
        comm.open_peers(handles)
        ok = True
    except Exception as e:  # noqa: BLE001
        ok, err = False, f"{type(e).__name__}: {e}"
    _log(f"setup: peers opened ({ok})")
    oks = _gather(ok, W)
    if not all(oks):
        info["peer"] = f"off: IPC open failed ({err or 'on another rank'})"
        comm.close()
        return None
    # a fabric that never delivers a flag costs the self-test one short bounded wait per call
    # (TDQ_PEER_SELFTEST_TIMEOUT_S), not the step-time bound, before every rank falls back
    ticks, comm.timeout_ticks = comm.timeout_ticks, int(float(os.environ.get("TDQ_PEER_SELFTEST_TIMEOUT_S", 5)) * 1e8)
    try:
        ok = _self_test(comm, min(comm.cap, bench_floats + 777))
    except Exception as e:  # noqa: BLE001
        ok, err = False, f"{type(e).__name__}: {e}"
    comm.timeout_ticks = ticks
    _log(f"setup: self-test {ok} err={err}")
    oks = _gather(ok, W)
    info["memory"] = _KINDS.get(comm.kind, "?")
    if not all(oks):
        info["peer"] = f"off: self-test failed ({err or 'wrong sums or a timeout'})"
        comm.close()
        return None
    # in-graph replay timings (how the step runs the collective); settle() re-decides at the
    # step's real bucket size once the engine knows it
    if m == "auto":
        t_peer, t_ref = _compare(comm, ctx, bench_floats)
    else:
        t_peer, t_ref = _time_us_graph(comm.all_reduce_, torch.randn(bench_floats, device=ctx.device), ctx), float("nan")
        t_peer = max(_gather(t_peer, W))
    _log(f"setup: peer {t_peer:.1f} us, torch.distributed {t_ref:.1f} us")
    info.update(peer_us=round(t_peer, 2), torch_us=None if t_ref != t_ref else round(t_ref, 2),
                bench_floats=bench_floats)
    use = m == "1" or not (t_ref <= t_peer)
    if comm.err.item() != 0:  # a late timeout during the timing
        use = False
    uses = _gather(use, W)
    if not all(uses):
        info["peer"] = "off: slower than torch.distributed" if all(not u for u in uses) else "off: disagreement"
        comm.close()
        return None
    info["impl"] = "peer one-shot"
    info["peer"] = "on"
    return comm
