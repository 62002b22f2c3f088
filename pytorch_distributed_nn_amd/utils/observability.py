"""Tracing, metrics and checkpointing.

* :class:`Tracer` — Chrome-trace JSON timeline (the reference's TF FULL_TRACE timeline,
  distributed_TF/src/distributed_train.py:284-310, and the C++ master's arrival timeline,
  MPI_code/.../sync_replicas_master_nn.h:61-63) with host spans for forward / backward / all-reduce /
  optimizer, plus roctx ranges (``torch.cuda.nvtx`` maps to roctx on ROCm) so the same phases appear in
  ``rocprofv3 --marker-trace``.
* :class:`MetricsSink` — one JSON record per step (step, loss, samples/s, phase ms, alive count).
* :func:`accuracy` — top-k precision (pytorch_code/nn_ops/__init__.py:13-26).
* :func:`save_checkpoint` / :func:`load_checkpoint` — ``{'epoch','arch','state_dict','best_prec1',
  'optimizer'}`` (the reference's sketch, backup/dist_nn_test.py:136-142) + step + RNG state; tensors are
  saved contiguous in torch layout so reference models load them; loading uses ``weights_only=True``.
"""
from __future__ import annotations

import contextlib
import json
import os
import threading
import time

import torch


class Tracer:
    def __init__(self, path: str | None = None, rank: int = 0, roctx: bool = True):
        self.path, self.rank = path, rank
        self.events = []
        self.roctx = roctx and torch.cuda.is_available()
        self._t0 = time.perf_counter()
        self._lock = threading.Lock()

    def _us(self):
        return (time.perf_counter() - self._t0) * 1e6

    @contextlib.contextmanager
    def span(self, name: str, cat: str = "step", sync: bool = False, **args):
        if self.roctx:
            torch.cuda.nvtx.range_push(name)
        if sync and torch.cuda.is_available():
            torch.cuda.synchronize()
        t = self._us()
        try:
            yield
        finally:
            if sync and torch.cuda.is_available():
                torch.cuda.synchronize()
            d = self._us() - t
            if self.roctx:
                torch.cuda.nvtx.range_pop()
            with self._lock:
                self.events.append({"name": name, "cat": cat, "ph": "X", "ts": t, "dur": d, "pid": self.rank,
                                    "tid": threading.get_ident() % 100000, "args": args})

    def instant(self, name: str, cat: str = "comm", args=None):
        with self._lock:
            self.events.append({"name": name, "cat": cat, "ph": "i", "s": "t", "ts": self._us(), "pid": self.rank,
                                "tid": threading.get_ident() % 100000, "args": args or {}})

    def save(self, path: str | None = None):
        path = path or self.path
        if not path:
            return None
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as f:
            json.dump({"traceEvents": self.events, "displayTimeUnit": "ms"}, f)
        return path


class MetricsSink:
    def __init__(self, path: str | None):
        self.path = path
        if path:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        self._f = open(path, "a") if path else None

    def log(self, **rec):
        rec.setdefault("time", time.time())
        if self._f:
            self._f.write(json.dumps(rec) + "\n")
            self._f.flush()
        return rec

    def close(self):
        if self._f:
            self._f.close()


def accuracy(output, target, topk=(1,)):
    """precision@k for the specified values of k (percent)."""
    maxk = max(topk)
    bs = target.size(0)
    _, pred = output.float().topk(maxk, 1, True, True)
    pred = pred.t()
    correct = pred.eq(target.view(1, -1).expand_as(pred))
    return [correct[:k].reshape(-1).float().sum(0).mul_(100.0 / bs) for k in topk]


def _plain_state_dict(module):
    sd = module.state_dict()
    return {k: v.detach().contiguous().clone().cpu() for k, v in sd.items()}


def save_checkpoint(path, model, optimizer=None, epoch=0, step=0, arch="", best_prec1=0.0, extra=None):
    m = model.module if hasattr(model, "module") else model
    ck = {"epoch": epoch, "step": step, "arch": arch, "state_dict": _plain_state_dict(m), "best_prec1": best_prec1,
          "rng": {"cpu": torch.get_rng_state(),
                  "cuda": torch.cuda.get_rng_state() if torch.cuda.is_available() else None}}
    if optimizer is not None:
        ck["optimizer"] = optimizer.state_dict()
    if extra:
        ck.update(extra)
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    tmp = path + ".tmp"
    torch.save(ck, tmp)
    os.replace(tmp, path)
    return path


def load_checkpoint(path, model, optimizer=None, map_location="cpu", restore_rng=True):
    """``path``: a checkpoint file (loaded with weights_only=True) or an already loaded checkpoint dict."""
    ck = path if isinstance(path, dict) else torch.load(path, map_location=map_location, weights_only=True)
    m = model.module if hasattr(model, "module") else model
    m.load_state_dict(ck["state_dict"])
    fp = getattr(m, "_pdnn_flat", None)
    if fp is not None:
        fp.refresh_shadow()
    if optimizer is not None and "optimizer" in ck:
        optimizer.load_state_dict(ck["optimizer"])
    if restore_rng and ck.get("rng"):
        torch.set_rng_state(ck["rng"]["cpu"])
        if ck["rng"].get("cuda") is not None and torch.cuda.is_available():
            torch.cuda.set_rng_state(ck["rng"]["cuda"])
    return ck
