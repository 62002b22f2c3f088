"""Training loop (PT-04 NN_Trainer, pytorch_code/nn_ops/__init__.py:28-85; single-machine baseline PT-07;
the DDP worker loop of PT-08; the TF trainer's examples/sec logging, distributed_train.py:315-321).

``Trainer(model, ...).train(loader)`` runs zero_grad -> forward -> loss -> backward (bucketed RCCL
all-reduce overlapped when the model is wrapped in our DDP) -> fused optimizer step, and logs one line per
``log_interval`` iterations in the reference's worker format, extended with samples/sec:

    Worker: 0, Train Epoch: 0 [128/60000 (0%)], Train Loss: 2.3026, Time Cost: 0.0120,
    FetchData: 0.0001, Forward: 0.0030, Backward: 0.0070, Step: 0.0010, Samples/s: 10666.7, Prec@1: 9.38

plus a JSONL metrics record per step and an optional Chrome-trace timeline.
"""
from __future__ import annotations

import time

import torch

from .ops import functional as OF
from .parallel.ddp import StepAborted
from .utils.observability import MetricsSink, Tracer, accuracy, load_checkpoint, save_checkpoint


class Trainer:
    def __init__(self, model, optimizer, loss_fn=None, device=None, rank=0, world=1, log_interval=10,
                 metrics_path=None, trace_path=None, checkpoint_dir=None, arch="", timing=True, printer=print,
                 lr_schedule=None, grad_clip=None, graph=False, graph_warmup=2, checkpoint_interval=0,
                 watchdog=None, compute_log=None):
        self.model = model
        self.opt = optimizer
        self.loss_fn = loss_fn or OF.cross_entropy
        self.device = device or torch.device("cpu")
        self.rank, self.world = rank, world
        self.log_interval = log_interval
        self.metrics = MetricsSink(metrics_path)
        self.tracer = Tracer(trace_path, rank) if trace_path else None
        self.checkpoint_dir = checkpoint_dir
        self.arch = arch
        self.timing = timing and self.device.type == "cuda"
        self.print = printer
        self.lr_schedule = lr_schedule
        self.grad_clip = grad_clip
        self.step_no = 0
        self.epoch = 0
        self.history = []
        self.checkpoint_interval = checkpoint_interval     # steps between rank-0 checkpoints (0: epoch ends)
        self.watchdog = watchdog                           # parallel.watchdog.CommWatchdog, fed every step
        # per-step compute-time records (TF-04 timeout_manager.py:48-70: dequeue / finish times per worker
        # and iteration), one JSONL per rank; tools/report.py cdf builds the CDF and p80/p90/p95/p99
        self.compute_log = MetricsSink(compute_log) if compute_log else None
        # hipGraph-captured step (utils/graphs.py): one replay per iteration instead of ~1000 launches
        self.graph_step = None
        if graph and self.device.type == "cuda":
            from .utils.graphs import GraphedStep
            self.graph_step = GraphedStep(model, optimizer, self.loss_fn, warmup=graph_warmup, grad_clip=grad_clip,
                                          allow_collectives=graph == "collectives")

    # ----------------------------------------------------------------------------------------- step
    def _mark(self):
        """A phase boundary: a timing event on the current stream (GPU: read lazily, the host never waits for
        it) or the host clock (CPU: the ops ran synchronously)."""
        if self.timing:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            return ev
        return time.perf_counter()

    @staticmethod
    def _phases(marks):
        """Phase durations (s) between consecutive marks; GPU events are waited for (only the last one)."""
        if isinstance(marks[0], float):
            return tuple(b - a for a, b in zip(marks, marks[1:]))
        marks[-1].synchronize()
        return tuple(a.elapsed_time(b) / 1e3 for a, b in zip(marks, marks[1:]))

    @staticmethod
    def _done(marks):
        return isinstance(marks[-1], float) or marks[-1].query()

    def _span(self, name):
        if self.tracer is None:
            import contextlib
            return contextlib.nullcontext()
        return self.tracer.span(name)

    def step(self, x, y):
        """One training iteration; returns (loss tensor, logits, phase marks).

        The marks are 4 phase boundaries (start, forward end, backward+all-reduce end, optimizer end): HIP
        events on a GPU, resolved into durations by :meth:`_phases` only when a record is written, so the host
        never synchronises inside the step and keeps running ahead of the device (the reference's per-phase
        Forward / Backward / Step fields, nn_ops/__init__.py:46-85; on a GPU they are device times)."""
        if self.lr_schedule is not None:
            for g in self.opt.param_groups:
                g["lr"] = self.lr_schedule(self.step_no)
        m0 = self._mark()
        if self.graph_step is not None:       # whole step is one graph: no per-phase split
            with self._span("graph_step"):
                loss = self.graph_step(x, y)
            m1 = self._mark()
            self.step_no += 1
            return loss, self.graph_step.output, (m0, m0, m1, m1)
        self.opt.zero_grad()
        kofn = getattr(self.model, "kofn", None) is not None
        with self._span("forward"):
            try:
                out = self.model(x)
                loss = self.loss_fn(out, y)
            except StepAborted:
                # k-of-n DDP closed this step during the forward: the wrapper already took part in the step's
                # collectives (zero contribution); no loss, no backward, the averaged gradient is applied below
                if not kofn:
                    raise
                out = loss = None
        m1 = self._mark()
        with self._span("backward+allreduce"):
            if loss is None:
                pass
            elif kofn:
                self.model.backward(loss)        # k-of-n DDP: a killed rank skips the rest of its backward
            else:
                loss.backward()
        m2 = self._mark()
        if self.grad_clip:
            if getattr(self.model, "_ovl_opt", None) is not None:
                # the optimizer already ran per bucket inside the backward (DistributedDataParallel.
                # overlap_optimizer): clipping now would be silently skipped
                raise ValueError("grad_clip cannot be combined with DistributedDataParallel.overlap_optimizer")
            torch.nn.utils.clip_grad_norm_(self.model.parameters(), self.grad_clip)
        with self._span("optimizer"):
            self.opt.step()
        m3 = self._mark()
        self.step_no += 1
        return loss, out, (m0, m1, m2, m3)

    # ----------------------------------------------------------------------------------------- loops
    def _finish(self, pend):
        """Write the per-step record of a step whose phase marks have resolved."""
        rec, marks, fetch, t_deq, bs = pend
        tfw, tbw, topt = self._phases(marks)
        total = fetch + tfw + tbw + topt
        rec.update(fetch_ms=1e3 * fetch, forward_ms=1e3 * tfw, backward_ms=1e3 * tbw, opt_ms=1e3 * topt,
                   samples_per_s=bs * self.world / max(total, 1e-9))
        self.metrics.log(**rec)
        self.history.append(rec)
        if self.compute_log is not None:
            self.compute_log.log(rank=self.rank, step=rec["step"], t_dequeue=t_deq, t_finish=t_deq + total,
                                 compute_ms=1e3 * (tfw + tbw + topt))
        return total

    def train(self, loader, epochs: int = 1, max_steps: int | None = None, steps_per_epoch: int | None = None,
              batch_size: int | None = None, dataset_size: int | None = None, skip_consumed: bool = True):
        from collections import deque
        n_per_epoch = steps_per_epoch or (len(loader) if hasattr(loader, "__len__") else 100)
        done = False
        # a resumed run continues at its checkpoint: `epoch` is the epoch in progress (epoch-end checkpoints
        # store the NEXT epoch), and a mid-epoch checkpoint resumes after the steps that epoch already ran
        first_i = max(0, self.step_no - self.epoch * n_per_epoch)
        # the loader is ONE stream across epochs (per-epoch reshuffles included) and a fresh loader restarts it
        # at its first batch: skip every batch the checkpointed run trained on -- all earlier epochs too, not
        # only this epoch's.  Loaders with skip() move only their sampler (no gather, no copy;
        # ADVICE r4), and the watchdog is fed meanwhile, so a long fast-forward is not taken for a hang.
        n_skip = self.step_no if skip_consumed else 0
        if n_skip and hasattr(loader, "skip"):
            loader.skip(n_skip)
            n_skip = 0
        it = iter(loader)
        for k in range(n_skip):
            next(it)
            if self.watchdog is not None and k % 64 == 0:
                self.watchdog.beat(self.step_no)
        pending = deque()          # steps whose phase events have not resolved yet (GPU), in step order
        for ep in range(self.epoch, epochs):
            self.epoch = ep
            start, first_i = (first_i if first_i < n_per_epoch else 0), 0
            for i in range(start, n_per_epoch):
                tf = time.perf_counter()
                x, y = next(it)
                if x.device != self.device:
                    x, y = x.to(self.device, non_blocking=True), y.to(self.device, non_blocking=True)
                fetch = time.perf_counter() - tf
                loss, out, marks = self.step(x, y)
                bs = x.shape[0]
                rec = {"step": self.step_no, "epoch": ep, "loss": None}
                pending.append((rec, marks, fetch, tf, bs))
                log_now = loss is not None and (self.step_no % self.log_interval == 0 or
                                                 (max_steps and self.step_no >= max_steps))
                if log_now:
                    lv = float(loss.detach())
                    if lv != lv or lv in (float("inf"), float("-inf")):      # TF trainer's NaN assert
                        raise FloatingPointError(f"Model diverged with loss = {lv} at step {self.step_no}")
                    p1 = float(accuracy(out.detach(), y, (1,))[0]) if out.dim() == 2 else float("nan")
                    rec["loss"], rec["prec1"] = lv, p1
                if log_now:          # once this step has completed on the device: a wall-clock point of the run
                    if not isinstance(marks[-1], float):
                        marks[-1].synchronize()
                    rec["wall_s"] = time.perf_counter()
                while pending and (log_now or self._done(pending[0][1])):
                    total = self._finish(pending.popleft())
                if log_now:
                    seen = (i + 1) * bs
                    tot = dataset_size or n_per_epoch * bs
                    self.print(f"Worker: {self.rank}, Train Epoch: {ep} [{seen}/{tot} ({100.0 * seen / tot:.0f}%)], "
                               f"Train Loss: {lv:.4f}, Time Cost: {total:.4f}, FetchData: {fetch:.4f}, "
                               f"Forward: {rec['forward_ms'] / 1e3:.4f}, Backward: {rec['backward_ms'] / 1e3:.4f}, "
                               f"Step: {rec['opt_ms'] / 1e3:.4f}, Samples/s: {rec['samples_per_s']:.1f}, "
                               f"Prec@1: {p1:.2f}")
                if self.watchdog is not None:
                    self.watchdog.beat(self.step_no)
                if (self.checkpoint_dir and self.checkpoint_interval and self.rank == 0
                        and self.step_no % self.checkpoint_interval == 0):
                    self.save(f"{self.checkpoint_dir}/checkpoint_step{self.step_no}.pt")
                if max_steps and self.step_no >= max_steps:
                    done = True
                    break
            if self.checkpoint_dir and self.rank == 0 and not done:
                self.epoch = ep + 1                   # the checkpoint resumes at the start of the next epoch
                self.save(f"{self.checkpoint_dir}/checkpoint_ep{ep}.pt")
            if done:
                break
        else:
            self.epoch = max(self.epoch, epochs)
        while pending:
            self._finish(pending.popleft())
        if self.tracer is not None:
            self.tracer.save()
        return self.history

    @torch.no_grad()
    def evaluate(self, loader, n_batches: int):
        self.model.eval()
        it = iter(loader)
        tot_loss, p1s, p5s, n = 0.0, 0.0, 0.0, 0
        for _ in range(n_batches):
            x, y = next(it)
            x, y = x.to(self.device), y.to(self.device)
            out = self.model(x)
            tot_loss += float(self.loss_fn(out, y)) * x.shape[0]
            k5 = min(5, out.shape[1])
            p1, p5 = accuracy(out, y, (1, k5))
            p1s += float(p1) * x.shape[0]
            p5s += float(p5) * x.shape[0]
            n += x.shape[0]
        self.model.train()
        res = {"loss": tot_loss / n, "prec1": p1s / n, "prec5": p5s / n}
        self.print(f"Test set: Average loss: {res['loss']:.4f}, Prec@1: {res['prec1']:.2f} Prec@5: {res['prec5']:.2f}")
        return res

    # ----------------------------------------------------------------------------------------- checkpoints
    def save(self, path, best_prec1=0.0):
        return save_checkpoint(path, self.model, self.opt, epoch=self.epoch, step=self.step_no, arch=self.arch,
                               best_prec1=best_prec1)

    def resume(self, path):
        """Restore model / optimizer / step / RNG from ``path`` (``"auto"``: the newest checkpoint in
        ``checkpoint_dir``, no-op when there is none — the restart-after-hang path of parallel/watchdog.py).

        With more than one rank, only rank 0 resolves and reads the checkpoint (checkpoint directories are
        written by rank 0 and need not be shared) and broadcasts it; every rank then loads the same model,
        optimizer state and step, so no rank continues with stale weights or an empty optimizer state."""
        import torch.distributed as dist
        multi = self.world > 1 and dist.is_available() and dist.is_initialized()
        ck = None
        if not multi or dist.get_rank() == 0:
            if path == "auto":
                from .parallel.watchdog import latest_checkpoint
                path = latest_checkpoint(self.checkpoint_dir)
            if path is not None:
                ck = torch.load(path, map_location="cpu", weights_only=True)
        if multi:
            box = [ck]
            dist.broadcast_object_list(box, src=0)
            ck = box[0]
        if ck is None:
            return None
        load_checkpoint(ck, self.model, self.opt, map_location=self.device, restore_rng=not multi)
        self.epoch, self.step_no = ck.get("epoch", 0), ck.get("step", 0)
        return ck
