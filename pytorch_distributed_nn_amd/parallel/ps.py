"""Parameter-server synchronous SGD with straggler mitigation — the reference's namesake capability.

Reference behaviour reproduced (defects of §2.11 fixed):

* roles: rank 0 = master (PT-02 SyncReplicasMaster_NN / CPP-03), optional rank 1 = evaluator (CPP-05,
  TF-06), the rest = workers (PT-03 DistributedWorker / CPP-04 WorkerNN).
* **layer-pipelined weight push** every step, in FORWARD bucket order (the reverse of the gradient
  buckets): ``comm_type="Bcast"`` — one broadcast per bucket of the flat fp32 weight arena from the
  master (reference: one MPI Bcast per parameter, sync_replicas_master_nn.py:259-272);
  ``comm_type="Async"`` — point-to-point sends of each bucket to each worker (reference Isend per
  parameter per worker, :243-257; the C++ master's per-layer Isend tagged with the step,
  MPI_code/src/distributed/sync_replicas_master_nn.h:193-211).  A worker posts every bucket's receive at
  once and a forward pre-hook on each module waits only for the bucket(s) holding that module's weights,
  so layer i computes while the weights of layers > i are still in flight (the C++ worker's
  ``MPI_Wait`` on layer i's request just before computing layer i, worker_nn.h:66-70).
* **optimizer parity**: the master applies the averaged gradient with the configured fused optimizer —
  SGD (momentum / weight decay), Adam or AdamW — and the TF trainer's exponential staircase LR decay
  (``lr * factor ** (step // decay_steps)``; distributed_TF/src/distributed_train.py:143-147,160-173; the
  wrapped optimizer applies the aggregated gradient, sync_replicas_optimizer_modified.py:363-410).
* **checkpointing on the master** (TF ``Supervisor(save_model_secs=...)`` plus the chief's final save,
  distributed_train.py:215-223,346-350): every ``save_model_secs`` of wall time and once at the end.
* **live compute-time side channel** (TF-04 TimeoutServer, timeout_manager.py:48-70,132-162): each
  worker's end-of-step marker carries its dequeue->finish compute time; the master logs the sorted
  per-step ELAPSED times of all workers while the run is in progress (``log_compute_times``) and keeps
  them in its per-step log.
* **gradient streaming per bucket**: the worker's gradient arena is cut into reverse-order buckets (the
  order backward produces them, as the DDP wrapper does); a post-accumulate-grad hook sends each bucket
  to the master the moment its last parameter is ready (reference: every parameter is Isent as soon as
  the layer-wise backward produced it, pytorch_code/model_ops/lenet.py:106-152, resnet_split.py:235-326,
  MPI_code/src/distributed/worker_nn.h:97-107).  Each send is announced as one entry
  ``rank,step,bucket`` in a global arrival queue in the control-plane store; the master consumes the
  queue in order with BLOCKING reads (no polling) — the store-side equivalent of the reference master's
  ``Irecv(ANY_SOURCE)`` + ``Waitany`` loop (sync_replicas_master_nn.py:150-206), and it works unchanged on
  gloo and on RCCL (whose p2p has no any-source receive).
* the master feeds every arrival to the C++ :class:`PSCoordinator` (per-bucket counts; full sync, k-of-n
  kill on the k-th arrival of the sentinel = the last bucket, i.e. parameter 0 as in the reference, or
  backup workers n_to_collect < n), accumulates only fresh gradients of the current step, divides every
  bucket by ITS count (fixes D3) and applies the update with the fused SGD kernel (optim.hip; momentum and
  weight decay honoured, fixes D9).  Once the step is closed, the buckets still in flight are received
  and DROPPED (CPP-03 drops gradients tagged with an old step, sync_replicas_master_nn.h:85): every
  worker ends its step with an end marker in the queue and the master drains up to the markers before
  the next weight push, so every p2p send is matched (a collective weight push must not wait on a send
  the master has not received).
* kill / short-circuit: when the master closes a step it publishes ``kill/<step>`` (the late workers,
  possibly none) in the store; a watcher thread per worker blocks on that key and raises a host flag,
  which the gradient hooks poll between buckets (an attribute read, no RPC).  A killed worker raises
  :class:`StepAborted` from the hook: autograd stops, so no further kernels are enqueued, and on GPU the
  host is kept at most two buckets ahead of the device so the flag reflects real GPU progress
  (reference busy-polls Iprobe(0, 77), lenet.py:168-178; short-circuit worker_nn.h:59-64,79-84).
* straggler injection: ``inject_straggler={rank: delay_ms}`` sleeps per parameter on those ranks
  (pure_py_code/distributed_worker.py:131-132's ``sleep(0.5)`` on ranks 1-3).
* interval mode (TF TimeoutReplicasOptimizer, sync_replicas_optimizer_modified.py:208-215): the timer
  runs from the moment the step is OPENED (the reference fires ``_update_op`` on a wall-clock timer
  regardless of arrivals); when it expires the step closes with what arrived, provided every bucket has
  at least one gradient (the reference's ``take_grad(1)`` blocks for one).  Arrivals after the close are
  dropped (the coordinator is closed too).
* evaluator: receives the weights (Bcast: joins the broadcast; Async: its own p2p copy) every
  ``eval_interval`` steps and appends ``step time_ms loss err`` to ``time_loss_out_<scheme>``.
"""
from __future__ import annotations

import json
import os
import threading
import time
from dataclasses import dataclass, field

import torch
import torch.distributed as dist

from ..ops.fused_resnet import side_stream_if_active
from ..optim.flat import ParamUseMode, flatten_module, register_grad_ready_hook, reverse_buckets
from ..utils.native import PSCoordinator, Store, StoreServer, StoreTimeout


class StepAborted(RuntimeError):
    """Raised inside a worker's backward to abandon a step (kill signal or a newer step)."""


class _StagedRecv:
    """irecv of a CUDA tensor over gloo through a host buffer (gloo's p2p moves host memory only).

    A reused host buffer (``host`` = a ``[buffer, event]`` pair owned by the caller) is not received into again
    until the asynchronous H2D copy of its previous contents has finished: the pair's event is recorded after
    that copy and waited on before the next irecv is posted."""

    def __init__(self, dst, src, host=None):
        self.dst = dst
        self.slot = host
        if host is not None:
            if host[1] is not None:
                host[1].synchronize()
            self.buf = host[0]
        else:
            self.buf = torch.empty(dst.shape, dtype=dst.dtype, pin_memory=True)
        self.work = dist.irecv(self.buf, src)

    def wait(self):
        self.work.wait()
        self.dst.copy_(self.buf, non_blocking=True)
        if self.slot is not None:
            ev = torch.cuda.Event()
            ev.record()
            self.slot[1] = ev


class _StagedSend:
    def __init__(self, src, dst):
        self.buf = src.detach().to("cpu")          # waits for the producing kernels
        self.work = dist.isend(self.buf, dst)

    def wait(self):
        self.work.wait()


def _nullcontext():
    import contextlib
    return contextlib.nullcontext()


@dataclass
class PSConfig:
    comm_type: str = "Bcast"          # "Bcast" | "Async"
    num_aggregate: int = 0            # k of k-of-n kill (0 = off)
    n_to_collect: int = 0             # backup-worker mode (0 = all workers)
    shortcircuit: bool = True
    interval_ms: float = 0.0          # >0: timer-driven step close (TF interval method)
    evaluator: bool = False           # rank 1 evaluates instead of training
    eval_interval: int = 10
    inject_straggler: dict = field(default_factory=dict)   # {rank: delay_ms per parameter}
    lr: float = 0.01
    momentum: float = 0.0
    weight_decay: float = 0.0
    optimizer: str = "sgd"            # "sgd" | "adam" | "adamw" (applied by the master)
    betas: tuple = (0.9, 0.999)
    eps: float = 1e-8
    lr_decay_factor: float = 1.0      # staircase decay: lr * factor ** (step // decay_steps)
    decay_steps: int = 0              # 0 = constant lr
    max_steps: int = 100
    out_dir: str = "outfiles"
    store_port: int = 0               # 0 = an ephemeral port chosen by the master's store and published to all ranks
    bucket_cap_mb: float = 4.0        # gradient streaming granularity
    first_bucket_mb: float = 0.25
    compute_times: bool = False       # workers write compute_times_rank<r>.jsonl (TF-04 side channel)
    log_compute_times: bool = False   # master prints the sorted per-step worker compute times (live)
    pipelined_push: bool = True       # per-bucket weight push + per-module waits (False: one transfer)
    push_delay_ms: float = 0.0        # fault injection: master pauses between weight buckets (slow link)
    checkpoint_dir: str = ""          # master checkpoints here every save_model_secs and at the end
    save_model_secs: float = 0.0


def make_optimizer(params, cfg: PSConfig):
    """The master's optimizer over the flat arena (fused kernel on GPU, torch reference on CPU)."""
    from ..optim import SGD, Adam, AdamW
    if cfg.optimizer == "sgd":
        return SGD(params, lr=cfg.lr, momentum=cfg.momentum, weight_decay=cfg.weight_decay)
    if cfg.optimizer == "adam":
        return Adam(params, lr=cfg.lr, betas=tuple(cfg.betas), eps=cfg.eps, weight_decay=cfg.weight_decay)
    if cfg.optimizer == "adamw":
        return AdamW(params, lr=cfg.lr, betas=tuple(cfg.betas), eps=cfg.eps, weight_decay=cfg.weight_decay)
    raise ValueError(f"PSConfig.optimizer: unknown optimizer {cfg.optimizer!r}")


def staircase_lr(cfg: PSConfig, step: int) -> float:
    """Learning rate of 1-based master step ``step`` (TF exponential_decay(staircase=True) of global_step =
    step - 1, distributed_train.py:143-147)."""
    if cfg.decay_steps <= 0 or cfg.lr_decay_factor == 1.0:
        return cfg.lr
    return cfg.lr * cfg.lr_decay_factor ** ((step - 1) // cfg.decay_steps)


def _start_control_plane(cfg: PSConfig):
    """Rank 0 starts the native control-plane store and every rank learns its port -> (server or None, port).

    The store binds ``cfg.store_port`` (0: the kernel picks a free port at bind time, so nothing can hold it
    already) and the real port travels to the other ranks over the process group that is already up.  The
    reference needs no port at all: its ranks find each other through MPI_COMM_WORLD
    (MPI_code/src/distributed_nn.cpp:16-24); a fixed ``MASTER_PORT + 1`` raced with gloo's own listeners."""
    server, err = None, ""
    if dist.get_rank() == 0:
        try:
            server = StoreServer(cfg.store_port)
        except OSError as e:          # still broadcast, so no rank is left waiting for the port
            err = str(e)
    box = [server.port if server is not None else -1, err]
    dist.broadcast_object_list(box, src=0)
    if box[0] < 0:
        raise OSError(f"parameter-server control plane did not start on rank 0: {box[1]}")
    return server, int(box[0])


class _Base:
    def __init__(self, model: torch.nn.Module, cfg: PSConfig, device):
        self.model = model
        self.cfg = cfg
        self.device = device
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()
        self.flat = flatten_module(model)
        self.buckets, self.pbucket = reverse_buckets(self.flat, cfg.bucket_cap_mb, cfg.first_bucket_mb)
        self.nb = len(self.buckets)
        self.first_worker = 2 if cfg.evaluator else 1
        self.workers = list(range(self.first_worker, self.world))
        self.n_workers = len(self.workers)
        self.scheme = (f"PS{cfg.comm_type}_k{cfg.num_aggregate}_collect{cfg.n_to_collect or self.n_workers}"
                       f"_of{self.n_workers}{'_shortcircuit' if cfg.shortcircuit else ''}")
        self._server, self.store_port = _start_control_plane(cfg)
        self.host = os.environ.get("MASTER_ADDR", "127.0.0.1")
        self.store = Store(self.host, self.store_port)
        self._pending, self._land = {}, {}

    # point-to-point transfers: direct on RCCL (and for host tensors); staged through host memory when CUDA
    # tensors travel over gloo (the one-GPU test boxes run several ranks on one device)
    def _staged(self, t):
        return t.is_cuda and dist.get_backend() == "gloo"

    def _isend(self, t, dst):
        return _StagedSend(t, dst) if self._staged(t) else dist.isend(t, dst)

    def _irecv(self, t, src, host=None):
        return _StagedRecv(t, src, host) if self._staged(t) else dist.irecv(t, src)

    def _recv(self, t, src):
        self._irecv(t, src).wait()

    def _weight_buckets(self):
        """Weight-push units in forward order: the gradient buckets reversed (one unit when not pipelined)."""
        if not self.cfg.pipelined_push:
            return [(-1, 0, self.flat.numel)]
        return [(b, s, e) for b, (s, e, _) in reversed(list(enumerate(self.buckets)))]

    def _push_weights(self, step: int):
        """Master: send the flat fp32 weight arena bucket by bucket in forward order, then wait."""
        works = []
        for i, (b, s, e) in enumerate(self._weight_buckets()):
            if self.cfg.push_delay_ms and i:
                time.sleep(self.cfg.push_delay_ms / 1e3)
            view = self.flat.data[s:e]
            if self.cfg.comm_type == "Bcast":
                works.append(dist.broadcast(view, 0, async_op=True))
            else:
                works += [self._isend(view, r) for r in range(1, self.world)]
        for w in works:
            w.wait()

    def _post_weight_recvs(self):
        """Receivers: post every bucket's receive at once -> {bucket: work}.  :meth:`_wait_bucket` completes
        one (and refreshes that slice of the bf16 shadow); nothing else blocks."""
        self._pending = {}
        self._land = {}
        for b, s, e in self._weight_buckets():
            view = self.flat.data[s:e]
            if self.cfg.comm_type == "Bcast":
                self._pending[b] = dist.broadcast(view, 0, async_op=True)
            else:
                self._pending[b] = self._irecv(view, 0)

    def _wait_bucket(self, b):
        w = self._pending.pop(b, None)
        if w is None:
            return
        w.wait()
        s, e = (0, self.flat.numel) if b < 0 else self.buckets[b][:2]
        self.flat.refresh_shadow_range(s, e)
        self._land[b] = time.perf_counter()

    def _wait_all_weights(self):
        for b in list(self._pending):
            self._wait_bucket(b)

    def close(self):
        dist.barrier()
        self.store.close()
        if self._server is not None:
            self._server.stop()


class PSMaster(_Base):
    """Rank 0: pushes weights, consumes the per-bucket arrival queue (k-of-n / backup / full sync /
    interval), averages each bucket by its count, applies the fused SGD update."""

    def __init__(self, model, cfg, device):
        super().__init__(model, cfg, device)
        # coordinator layers = buckets in reverse, so layer 0 is the LAST bucket (parameter 0: the sentinel)
        self.coord = PSCoordinator(self.n_workers, self.nb, cfg.n_to_collect, cfg.num_aggregate)
        self.opt = make_optimizer(self.flat.params, cfg)
        # one staging slot per (worker, bucket), allocated on first use and reused every step: a receive is
        # posted the moment its arrival is announced, so the transfers of all workers overlap.  Memory: one fp32
        # copy of the model per worker on the master's device (plus a pinned host copy when CUDA tensors travel
        # over gloo) -- ~0.8 GB for ResNet-50 at 8 workers, well inside one MI355X's 288 GB (the reference
        # pre-posts P x (N-1) Irecv(ANY_SOURCE) and Waitany's over them, sync_replicas_master_nn.py:143-150,
        # 275-284; the C++ master 100 per layer, sync_replicas_master_nn.h:163-186)
        self._slots = {}
        self.qpos = 0                          # next arrival-queue entry to read
        self.log = []
        self.store.set("scheme", self.scheme)

    def _next_arrival(self, timeout_ms):
        """(worker rank, step, bucket, compute_ms) of the next queued send, or None on timeout."""
        try:
            v = self.store.get(f"q/{self.qpos + 1}", timeout_ms=timeout_ms)
        except StoreTimeout:
            return None
        self.qpos += 1
        self.store.delete(f"q/{self.qpos}")
        f = v.decode().split(",")
        # end-of-step markers carry the worker's compute time (live TF-04 side channel) as a 4th field
        return int(f[0]), int(f[1]), int(f[2]), (float(f[3]) if len(f) > 3 else None)

    def _post_receive(self, r, b):
        """Post the receive of worker r's bucket b into its staging slot -> (slot, work)."""
        slot = self._slots.get((r, b))
        if slot is None:
            s, e, _ = self.buckets[b]
            dev = torch.zeros(e - s, dtype=torch.float32, device=self.flat.grad.device)
            host = [torch.empty(e - s, dtype=torch.float32, pin_memory=True), None] if self._staged(dev) else None
            slot = self._slots[(r, b)] = (dev, host)
        return slot[0], self._irecv(slot[0], r, slot[1])

    def _save(self, step, final=False):
        from ..utils.observability import save_checkpoint
        name = "checkpoint_final.pt" if final else f"checkpoint_step{step}.pt"
        path = save_checkpoint(os.path.join(self.cfg.checkpoint_dir, name), self.model, self.opt, step=step,
                               extra={"scheme": self.scheme})
        self.saved.append((step, path))
        return path

    def train(self):
        cfg = self.cfg
        t0 = time.perf_counter()
        self.saved = []
        last_save = t0
        for step in range(1, cfg.max_steps + 1):
            self.store.set_int(f"go/{step}", step)              # step broadcast (C-01 / C-08)
            self._push_weights(step)                            # C-02 / C-03, layer-pipelined
            self.coord.begin_step(step)
            self.flat.grad.zero_()
            tstep = time.perf_counter()
            closed, stale, ended = False, 0, set()
            ctimes = {}
            inflight = []                                       # posted receives, in announcement order
            xfer_ms = []                                        # per receive: post -> landed (overlapping)

            def take(timeout):
                """Post a receive for every arrival announced so far (non-blocking queue reads; blocking up to
                ``timeout`` only when nothing is in flight), then complete the oldest receive in flight and
                offer it to the coordinator: all announced transfers run concurrently."""
                nonlocal closed, stale
                got = False
                while True:
                    a = self._next_arrival(0 if (inflight or got) else timeout)
                    if a is None:
                        break
                    got = True
                    r, s, b, cms = a
                    if b < 0:                                   # end-of-step marker of worker r
                        if s == step:
                            ended.add(r)
                            ctimes[r] = cms
                        continue
                    g, work = self._post_receive(r, b)
                    inflight.append((r, s, b, g, work, time.perf_counter()))
                if not inflight:
                    return
                r, s, b, g, work, tpost = inflight.pop(0)
                work.wait()
                xfer_ms.append((time.perf_counter() - tpost) * 1e3)
                tms = (time.perf_counter() - t0) * 1e3
                res = self.coord.offer(self.workers.index(r), self.nb - 1 - b, s, tms)
                if res == PSCoordinator.ACCEPTED:
                    bs, be, _ = self.buckets[b]
                    self.flat.grad[bs:be].add_(g)
                elif res == PSCoordinator.STALE:
                    stale += 1
                if self.coord.done():
                    closed = True

            while not closed and (len(ended) < self.n_workers or inflight):
                timeout = -1
                if cfg.interval_ms:
                    rest = cfg.interval_ms - (time.perf_counter() - tstep) * 1e3
                    timeout = max(1, int(rest)) if rest > 0 else 1
                take(timeout)
                if (not closed and cfg.interval_ms and (time.perf_counter() - tstep) * 1e3 >= cfg.interval_ms
                        and all(self.coord.count(li) >= 1 for li in range(self.nb))):
                    closed = True
            self.coord.close()                                  # later arrivals of this step are dropped
            gather_ms = (time.perf_counter() - tstep) * 1e3
            # workers that did not deliver every bucket are killed (C-06, tag 77); published always so
            # every worker's watcher wakes for this step
            late = [w for i, w in enumerate(self.workers)
                    if not all(self.coord.contributed(li, i) for li in range(self.nb))]
            self.store.set(f"kill/{step}", json.dumps(late))
            while len(ended) < self.n_workers or inflight:     # receive (and drop) the late buckets, so
                take(-1)                                        # every p2p send of the step is matched
            # count-correct per-bucket average (fixes D3) + fused SGD (momentum, wd: fixes D9)
            counts = [self.coord.count(self.nb - 1 - b) for b in range(self.nb)]
            for b, (bs, be, _) in enumerate(self.buckets):
                if counts[b] > 1:
                    self.flat.grad[bs:be].mul_(1.0 / counts[b])
            lr = staircase_lr(cfg, step)
            for g in self.opt.param_groups:
                g["lr"] = lr
            self.opt.step()
            arrived = [w for i, w in enumerate(self.workers)
                       if all(self.coord.contributed(li, i) for li in range(self.nb))]
            elapsed = sorted(v for v in ctimes.values() if v is not None)
            self.log.append({"step": step, "arrived": arrived, "count": min(counts), "bucket_counts": counts,
                             "stale_dropped": stale, "gather_ms": gather_ms, "lr": lr, "compute_ms": elapsed,
                             "xfer_ms_sum": sum(xfer_ms), "receives": len(xfer_ms)})
            if cfg.log_compute_times:      # timeout_manager.py:48-70 "ELAPSED TIMES" line, live
                print(f"Master: step {step} ELAPSED TIMES (ms, sorted over workers) "
                      f"{[round(v, 2) for v in elapsed]}", flush=True)
            if cfg.checkpoint_dir and cfg.save_model_secs > 0 and time.perf_counter() - last_save >= cfg.save_model_secs:
                self._save(step)
                last_save = time.perf_counter()
        self.store.set_int(f"go/{cfg.max_steps + 1}", -1)
        self._push_weights(cfg.max_steps + 1)       # final weights, so evaluator/workers end consistent
        if cfg.checkpoint_dir:                      # the chief's final save (distributed_train.py:346-350)
            self._save(cfg.max_steps, final=True)
        os.makedirs(cfg.out_dir, exist_ok=True)
        with open(os.path.join(cfg.out_dir, f"timeline_out_{self.scheme}"), "w") as f:
            for t, s, w, li in self.coord.timeline():      # time_ms step worker bucket (arrival timeline)
                f.write(f"{t:.3f} {s} {self.workers[w]} {self.nb - 1 - li}\n")
        return self.log


class PSWorker(_Base):
    """Worker: receive weights, compute a gradient on its next batch, stream it to the master bucket by
    bucket; abort the backward when killed (short-circuit)."""

    def __init__(self, model, cfg, device, loss_fn):
        super().__init__(model, cfg, device)
        self.loss_fn = loss_fn
        self.delay = cfg.inject_straggler.get(self.rank, 0) / 1e3
        self._killable = bool(cfg.num_aggregate or cfg.interval_ms
                              or (cfg.n_to_collect and cfg.n_to_collect < self.n_workers))
        self.cur = 0
        self.abort_step = -1
        self.done_step = 0
        self._in_step = self._fwd_phase = self._aborted = False
        self.abort_phase = None
        self.step_end = None                # optional callable(worker, step, x, y) after a completed backward
        self._hooks = [register_grad_ready_hook(p, self._param_done) for p in self.flat.params]
        self._fwd_hooks = self._install_weight_waits()
        self.fwd_start = {}                 # step -> time the first module's forward began (timeline)
        self.landed = {}                    # step -> {weight bucket: time its receive completed}
        self.aborted_steps = 0
        self.compute_records = []
        self.sent = []                      # (step, bucket) in send order (tests / timeline)
        self._stop = False
        self.wstore = Store(self.host, self.store_port)     # the watcher's own connection
        from .ddp import warm_abort_path
        warm_abort_path(StepAborted)        # the first exception through autograd costs ~0.3 s once
        self._watcher = threading.Thread(target=self._watch, daemon=True)
        self._watcher.start()

    def _install_weight_waits(self):
        """Per-parameter hooks run before each use of a parameter in the forward:

        * the wait for the weight bucket that holds it and nothing else (pipelined push; the C++ worker's
          per-layer MPI_Wait just before computing the layer, worker_nn.h:66-70);
        * the forward-phase short-circuit: a worker the master has killed abandons the step before its next
          layer (the C++ worker checks before EVERY forward layer as well as every backward layer,
          worker_nn.h:56-64,77-84).

        A use is (a) the bf16 shadow fetch of every fused GPU op (``weight_bf16`` calls
        :func:`~..optim.flat.await_param`), and (b) any torch op taking the parameter as an argument, caught
        by :class:`~..optim.flat.ParamUseMode` around the worker's forward."""
        if not (self.cfg.pipelined_push or self.cfg.shortcircuit or self.cfg.num_aggregate):
            return []
        for p in self.flat.params:
            p._pdnn_await = self._before_param
            p._pdnn_weight_pending = True     # weights arrive during the forward: no early fp8 re-quantisation
        return list(self.flat.params)

    def _check_armed(self):
        return bool(self._pending) or self.abort_step == self.cur

    def _before_param(self, p):
        if self._in_step and self.abort_step == self.cur and not self._aborted:
            self._aborted = True
            self.abort_phase = "forward" if self._fwd_phase else "backward"
            raise StepAborted(f"rank {self.rank} step {self.cur} (before a layer)")
        b = self.pbucket.get(id(p))
        if b is None or b not in self._pending:
            return
        if self.cur not in self.fwd_start:
            self.fwd_start[self.cur] = time.perf_counter()
        self._wait_bucket(b)

    def _watch(self):
        # blocks on each step's kill key in turn (always published when the master closes the step)
        step = 1
        while not self._stop:
            try:
                v = self.wstore.get(f"kill/{step}", timeout_ms=500)
            except StoreTimeout:
                continue
            except Exception:
                return
            if (self.cfg.shortcircuit or self.cfg.num_aggregate) and self.rank in json.loads(v.decode()) \
                    and self.done_step < step:
                self.abort_step = step
            step += 1

    def _param_done(self, p):
        if self.delay:
            time.sleep(self.delay)                      # straggler injection, per parameter
        if self._aborted:
            return
        if self.abort_step == self.cur:                 # killed: skip the rest of the backward
            self._aborted = True
            self.abort_phase = "backward"
            raise StepAborted(f"rank {self.rank} step {self.cur}")
        b = self.pbucket[id(p)]
        self._ready[b] += 1
        while self._next < self.nb and self._ready[self._next] == self.buckets[self._next][2]:
            self._send(self._next)
            self._next += 1

    def _send(self, b):
        s, e, _ = self.buckets[b]
        view = self.flat.grad[s:e]
        if view.is_cuda and self._killable:
            # keep the host at most two buckets ahead of the GPU so a kill stops real GPU work.  Only where a
            # kill can happen (k-of-n, backup workers, interval close): under full sync no worker is ever cut
            # short, and the wait would only hold the host back.  The event is on the compute stream, as in
            # DistributedDataParallel._launch (the side stream lags by design).
            if len(self._events) >= 2:
                self._events[-2].synchronize()
            ev = torch.cuda.Event()
            ev.record()
            self._events.append(ev)
        self.store.push("q", f"{self.rank},{self.cur},{b}")        # one round trip (arrival queue)
        side = side_stream_if_active(view)
        if side is None:
            self._works.append(self._isend(view, 0))
        else:
            # fused ResNet blocks leave their weight gradients on the side stream (the hook is side-aware, so
            # the block does not join it before announcing them): the send is ordered after both streams
            from ..ops import kernels as K
            K.stream_wait(side, torch.cuda.current_stream(side.device))
            with torch.cuda.stream(side):
                self._works.append(self._isend(view, 0))
        self.sent.append((self.cur, b))

    def train(self, batches):
        it = iter(batches)
        while True:
            s = self.store.get_int(f"go/{self.cur + 1}")      # blocks until the master opens the step
            self._post_weight_recvs()                         # every bucket in flight; layers wait per bucket
            if not self.cfg.pipelined_push or s == -1:
                self._wait_all_weights()
            if s == -1:
                break
            self.cur = s
            t_deq = time.perf_counter()                       # step dequeued (TF-04 "worker_dequeued_token")
            x, y = next(it)
            self.flat.zero_grad()
            self._ready, self._next, self._works, self._events, self._aborted = [0] * self.nb, 0, [], [], False
            self.abort_phase = None
            self._in_step = True
            try:
                self._fwd_phase = True
                with ParamUseMode(self._check_armed) if self._fwd_hooks else _nullcontext():
                    out = self.model(x.to(self.device))
                self._fwd_phase = False
                self._wait_all_weights()                      # buckets no module claimed (and the backward's)
                self.landed[s] = dict(self._land)
                loss = self.loss_fn(out, y.to(self.device))
                loss.backward()
                self.done_step = s
                if self.step_end is not None:
                    self.step_end(self, s, x, y)
            except StepAborted:
                self.aborted_steps += 1
                self._wait_all_weights()        # a forward abort leaves weight receives posted: complete them
            finally:
                self._in_step = self._fwd_phase = False
            self.compute_records.append({"rank": self.rank, "step": s, "t_dequeue": t_deq,
                                         "t_finish": time.perf_counter(), "aborted": self.done_step != s,
                                         "abort_phase": self.abort_phase,
                                         "compute_ms": 1e3 * (time.perf_counter() - t_deq)})
            # end-of-step marker: the master drains this worker's sends up to it (late ones are dropped); it
            # carries the dequeue -> finish compute time, the master's live per-step ELAPSED TIMES
            self.store.push("q", f"{self.rank},{s},-1,{self.compute_records[-1]['compute_ms']:.4f}")
            for w in self._works:
                w.wait()
        self._stop = True
        if self.cfg.compute_times:
            os.makedirs(self.cfg.out_dir, exist_ok=True)
            with open(os.path.join(self.cfg.out_dir, f"compute_times_rank{self.rank}.jsonl"), "w") as f:
                for r in self.compute_records:
                    f.write(json.dumps(r) + "\n")
        return self.aborted_steps

    def close(self):
        self._stop = True
        super().close()
        # the watcher may be inside a blocking get on its connection: let it leave before freeing it
        self._watcher.join(timeout=5.0)
        if not self._watcher.is_alive():
            self.wstore.close()


class PSEvaluator(_Base):
    """Rank 1 (optional): evaluates the pushed weights; writes ``time_loss_out_<scheme>``
    (evaluator_nn.h:55-58 format: step time_ms loss err_rate)."""

    def __init__(self, model, cfg, device, eval_fn):
        super().__init__(model, cfg, device)
        self.eval_fn = eval_fn

    def train(self):
        os.makedirs(self.cfg.out_dir, exist_ok=True)
        path = os.path.join(self.cfg.out_dir, f"time_loss_out_{self.scheme}")
        t0 = time.perf_counter()
        rows = []
        cur = 0
        with open(path, "w") as f:
            while True:
                s = self.store.get_int(f"go/{cur + 1}")
                cur += 1
                self._post_weight_recvs()
                self._wait_all_weights()
                final = s == -1
                if final or s % self.cfg.eval_interval == 0:
                    loss, err = self.eval_fn(self.model)
                    step = self.cfg.max_steps if final else s
                    rows.append((step, (time.perf_counter() - t0) * 1e3, loss, err))
                    f.write(f"{step} {rows[-1][1]:.3f} {loss:.6f} {err:.6f}\n")
                    f.flush()
                if final:
                    break
        return rows


def run_ps(model, cfg: PSConfig, device, loss_fn=None, batches=None, eval_fn=None):
    """Dispatch by rank.  Returns the role-specific log."""
    rank = dist.get_rank()
    if rank == 0:
        role = PSMaster(model, cfg, device)
        out = role.train()
    elif cfg.evaluator and rank == 1:
        role = PSEvaluator(model, cfg, device, eval_fn)
        out = role.train()
    else:
        role = PSWorker(model, cfg, device, loss_fn)
        out = role.train(batches)
    role.close()
    return out


PSWorker._param_done._pdnn_side_aware = True      # _send orders each bucket after the weight-gradient stream
