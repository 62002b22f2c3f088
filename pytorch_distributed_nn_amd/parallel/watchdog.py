"""Hang detection and restart-from-checkpoint recovery for collective training (SURVEY.md §5.3 item 5:
"for true hangs: a watchdog calls ncclCommAbort, then re-initializes the communicator from the store
(restart-from-checkpoint recovery)").

The reference has no recovery at all: a dead or wedged rank stalls every MPI ``Waitany`` forever
(pytorch_code/sync_replicas_master_nn.py:148-150; MPI_code/src/distributed/sync_replicas_master_nn.h:66-74),
and its only liveness mechanism is the RPC side-channel's 30 s timeout (distributed_TF/src/
timeout_manager.py:79-105).  A collective cannot be cancelled, so here recovery is process-level:

1. :class:`CommWatchdog` is a host thread fed by a heartbeat — ``beat()`` after every completed step.  If
   no beat arrives within ``timeout_s`` the step is declared hung.
2. It writes a JSON record (rank, step, seconds since the last beat, Python stacks of every thread) to
   ``<dir>/hang_rank<r>.json``, aborts the process group (``ProcessGroupNCCL.abort()`` = ncclCommAbort on
   RCCL, so the peers' pending collectives fail instead of waiting) and ends the process with exit code
   :data:`EXIT_HANG`.
3. The launcher restarts the worker group (``torchrun --max-restarts N``; every rank re-runs rendezvous and
   builds a fresh communicator), and :meth:`Trainer.resume` / :func:`latest_checkpoint` continue from the
   newest checkpoint that rank 0 wrote (``--checkpoint-dir`` + ``--checkpoint-interval``, ``--resume auto``).

Exiting is deliberate: a rank whose HIP stream is stuck inside an RCCL kernel cannot be unstuck from
Python, and a half-aborted communicator must not be reused.
"""
from __future__ import annotations

import glob
import json
import os
import sys
import threading
import time
import traceback

EXIT_HANG = 75          # EX_TEMPFAIL: "try again" — the launcher's restart policy handles it


def _abort_process_group():
    try:
        import torch.distributed as dist
        if not dist.is_initialized():
            return "not initialised"
        pg = dist.distributed_c10d._get_default_group()
        be = dist.get_backend(pg)
        if be == "nccl":
            try:
                pg._get_backend(__import__("torch").device("cuda")).abort()      # ncclCommAbort
                return "nccl abort"
            except Exception as e:                                               # noqa: BLE001
                return f"nccl abort failed: {e!r}"
        return f"{be}: no abort (process exit ends its sockets)"
    except Exception as e:                                                       # noqa: BLE001
        return f"abort failed: {e!r}"


class CommWatchdog:
    """``wd = CommWatchdog(timeout_s=300).start(); ...; wd.beat(step)`` in the training loop."""

    def __init__(self, timeout_s: float = 600.0, out_dir: str | None = None, rank: int | None = None,
                 exit_on_hang: bool = True, on_hang=None, poll_s: float | None = None):
        self.timeout_s = float(timeout_s)
        self.out_dir = out_dir
        if rank is None:
            from .runtime import rank as _rank
            rank = _rank()
        self.rank = rank
        self.exit_on_hang = exit_on_hang
        self.on_hang = on_hang
        self.poll_s = poll_s if poll_s is not None else max(0.05, min(5.0, self.timeout_s / 10))
        self.step = -1
        self._last = time.monotonic()
        self._stop = threading.Event()
        self._thread = None
        self.fired = None

    def start(self):
        self._last = time.monotonic()
        self._thread = threading.Thread(target=self._run, name="pdnn-comm-watchdog", daemon=True)
        self._thread.start()
        return self

    def beat(self, step: int | None = None):
        self.step = self.step + 1 if step is None else step
        self._last = time.monotonic()

    def stop(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()

    # --------------------------------------------------------------------------------------------------
    def _record(self, idle):
        rec = {"rank": self.rank, "step": self.step, "idle_s": round(idle, 3), "timeout_s": self.timeout_s,
               "time": time.time(), "pid": os.getpid(),
               "stacks": {str(t): "".join(traceback.format_stack(f)) for t, f in sys._current_frames().items()}}
        return rec

    def _run(self):
        while not self._stop.wait(self.poll_s):
            idle = time.monotonic() - self._last
            if idle < self.timeout_s:
                continue
            rec = self._record(idle)
            rec["abort"] = _abort_process_group()
            self.fired = rec
            if self.out_dir:
                os.makedirs(self.out_dir, exist_ok=True)
                with open(os.path.join(self.out_dir, f"hang_rank{self.rank}.json"), "w") as f:
                    json.dump(rec, f)
            print(f"[watchdog] rank {self.rank}: no step completed for {idle:.1f}s (step {self.step}); "
                  f"{rec['abort']}; exiting with {EXIT_HANG} for a launcher restart", file=sys.stderr, flush=True)
            if self.on_hang is not None:
                self.on_hang(rec)
            if self.exit_on_hang:
                os._exit(EXIT_HANG)
            return


def latest_checkpoint(directory: str | None):
    """Newest ``*.pt`` checkpoint in ``directory`` (by mtime, then the number in its name), or None."""
    if not directory or not os.path.isdir(directory):
        return None
    files = glob.glob(os.path.join(directory, "*.pt"))
    if not files:
        return None

    def key(p):
        base = os.path.basename(p)
        num = "".join(ch if ch.isdigit() else " " for ch in base).split()
        return (os.path.getmtime(p), int(num[-1]) if num else -1)
    return max(files, key=key)
