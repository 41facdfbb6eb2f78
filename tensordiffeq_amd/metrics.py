"""JSONL training metrics (SURVEY.md §5 "Metrics / logging / observability").

The reference only shows tqdm postfixes and keeps symbolic loss tensors (B16).  Here every
``log_every`` steps one JSON object per line is appended: phase, epoch, total + per-term loss,
collocation-points/s and ms/step over the interval, rank.  Loss values come from the on-device
history buffer (one small D2H copy per interval, no extra sync inside the graph-captured steps).
"""
from __future__ import annotations

import json
import os
import time


class MetricsLogger:
    def __init__(self, path, rank=0, world=1, n_points=None):
        if world > 1:
            root, ext = os.path.splitext(path)
            path = f"{root}.rank{rank}{ext or '.jsonl'}"
        self.path = path
        self.rank, self.world, self.n_points = rank, world, n_points
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)
        self._f = open(path, "a", buffering=1)
        self._t = time.perf_counter()
        self._last = None

    def mark(self, epoch):
        self._t = time.perf_counter()
        self._last = epoch

    def log(self, phase, epoch, loss, terms=None, **extra):
        now = time.perf_counter()
        rec = {"phase": phase, "epoch": int(epoch), "loss": float(loss), "rank": self.rank,
               "world": self.world, "time": time.time()}
        if terms:
            rec["terms"] = {k: float(v) for k, v in terms.items()}
        if self._last is not None and epoch > self._last:
            dt = now - self._t
            steps = epoch - self._last
            rec["ms_per_step"] = 1e3 * dt / steps
            if self.n_points:
                rec["pts_per_s"] = self.n_points * self.world * steps / dt
        rec.update(extra)
        self._f.write(json.dumps(rec) + "\n")
        self._t, self._last = now, epoch
        return rec

    def log_event(self, event, **fields):
        """One non-periodic record (e.g. why L-BFGS stopped)."""
        rec = {"event": event, "rank": self.rank, "world": self.world, "time": time.time()}
        rec.update(fields)
        self._f.write(json.dumps(rec) + "\n")
        return rec

    def close(self):
        if self._f:
            self._f.close()
            self._f = None


def read_jsonl(path):
    with open(path) as f:
        return [json.loads(line) for line in f if line.strip()]
