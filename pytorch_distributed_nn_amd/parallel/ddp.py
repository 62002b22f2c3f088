"""DistributedDataParallel over RCCL (xGMI) — the north-star primitive (SURVEY.md §2.6 PAR-DP-ALLREDUCE,
§3.3; reference fork: pytorch_code/data_parallel_dist/data_parallel_dist.py:29-267).

What it does, and how it differs from the reference's design:

* **Init broadcast** of all parameters and buffers from rank 0 as ONE collective over the flat parameter
  arena (+ one coalesced broadcast of buffers) — the reference issues one broadcast per tensor
  (data_parallel_dist.py:45-46).
* **Buckets are zero-copy views** of the flat fp32 gradient buffer (``optim.FlatParams``), assigned in
  **reverse** parameter order (the order gradients are produced in backward), with a small first bucket
  so communication starts as early as possible.  The reference fills ~1 MB buckets in *forward* order
  and flattens/copies each one (defect D11; data_parallel_dist.py:70-83, 247, 262-263).
* **Overlap without Python threads**: a post-accumulate-grad hook counts ready parameters; when a
  bucket is complete its ``all_reduce`` is issued immediately (asynchronously, RCCL runs it on its own
  HIP stream ordered after the compute stream), strictly in bucket order so every rank issues the same
  collective sequence.  An autograd end-of-backward callback launches any remaining buckets (unused
  parameters) and waits.  The reference spawns one reduction thread + one process group per bucket
  (data_parallel_dist.py:211-267).
* **Averaging** uses RCCL's native AVG reduction (one pass, no extra scale kernel); on gloo (CPU) it is
  SUM followed by a scale.
* **Bucket sizing for xGMI** (default 32 MiB, the first bucket too: ``first_bucket_cap_mb`` may make it smaller).  A ring all-reduce of S bytes
  over N ranks costs T(S) ~= a + 2(N-1)/N * S / B, with a the per-collective latency and B the per-rank bus
  bandwidth.  Measured here (profiles/rccl_world1_r4.txt, device events, RCCL AVG): a ~= 12-18 us (the
  64 KiB-4 MiB sizes all take 13-18 us), and the world-1 reduction kernel itself runs at ~700 GB/s fp32, so it
  never binds.  At N = 8 each MI355X reaches its peers over 7 point-to-point xGMI links (~153 GB/s each per
  direction); a ring is bound by one link per hop, so B ~= 150-300 GB/s depending on how many channels RCCL
  spreads over the links.  Then a 32 MiB bucket takes ~= 15 + 1.75 * 33.5 MB / 200 GB/s ~= 310 us, latency
  is < 5% of it, and ResNet-50's 102 MB of fp32 gradients is 4 collectives (+ the small first one) ~= 1.2 ms of
  link time, against a ~15 ms backward that produces the buckets 1.3, 2.6, 5.7 and 15.7 ms after the first
  gradient hook (bench.py ``comm`` block): every bucket but the last is hidden under the backward.  What is
  exposed is the LAST bucket (stem + stage-1 parameters, 12.3 MiB, ready only when the backward ends): ~120 us
  at N = 8 by the model above.  Smaller buckets would not shrink it (those parameters' gradients all arrive in
  the backward's last ~1 ms) and would multiply the latency term; larger ones would delay the earlier buckets
  past the point where they overlap.  A small first bucket (PyTorch's 1 MiB) would hold only fc.bias here (the
  8 MB fc.weight does not fit) and start nothing useful early, while every collective also costs its issuing
  stream ~21 us (ProcessGroupNCCL's stream-sync event, gpurun_out/r5_40-44): the first bucket takes the full cap.
  Re-derive with ``tools/bench_allreduce.py`` at the real N.
* **k-of-n straggler kill / backup workers in collective form** (PAR-DP-KILL / PAR-DP-BACKUP, SURVEY.md
  §5.3; reference: pytorch_code/sync_replicas_master_nn.py:172-186 kill on the k-th arrival,
  pytorch_code/model_ops/lenet.py:168-178 worker poll, MPI_code/src/distributed/worker_nn.h:59-84
  short-circuit).  ``num_aggregate=k``: every rank reports "backward done" to the control-plane store
  (an atomic counter per step); the k-th reporter closes the step (``deadline_ms``: rank 0 also closes it
  when the deadline passes — the backup-worker / interval form).  A watcher thread per rank blocks on
  the close key and raises a host flag; the gradient hooks poll that flag (a Python attribute, no RPC)
  and a rank that is still computing abandons the rest of its backward (``StepAborted`` stops autograd,
  so no further kernels are enqueued; on GPU the host is kept at most two buckets ahead of the device so
  the decision reflects real GPU progress; with no straggler the whole machinery costs < 1% of a ResNet-50
  step, profiles/kofn_tax_r4.txt).  Collectives must stay matched, so the aborted rank still
  all-reduces every remaining bucket, zero-filled.  Each rank records per bucket whether it sent real
  gradients; that contribution vector is all-reduced after the buckets and every bucket is divided by
  ITS count — the count-correct average of the C++ master (sync_replicas_master_nn.h:125) per bucket,
  like the reference's per-parameter counters (sync_replicas_master_nn.py:30-79), fixing defect D3.
  ``straggler_mode`` alone keeps the manual form (``set_alive``).
* Optional **bf16 gradient compression** on the wire (``comm_dtype=torch.bfloat16``).
"""
from __future__ import annotations

import contextlib
import os
import time

import torch
import torch.distributed as dist
import torch.nn as nn

from ..ops.fused_resnet import side_stream_if_active
from ..optim.flat import ParamUseMode, flatten_module, register_grad_ready_hook, reverse_buckets


class StepAborted(RuntimeError):
    """Raised inside a rank's backward to abandon the rest of the step (k-of-n kill / short-circuit)."""


class _KofN:
    """Control plane of the k-of-n step close: two TCPStore clients on the rendezvous store (MASTER_ADDR /
    MASTER_PORT) — one for the main thread's reports, one blocked in `wait` by the watcher thread."""

    _instances = 0            # same construction order on every rank -> same key namespace

    def __init__(self, ddp, k: int, deadline_ms: float):
        import threading
        from datetime import timedelta
        self.ddp, self.k, self.deadline_ms = ddp, k, deadline_ms
        host = os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = int(os.environ.get("MASTER_PORT", "29500"))
        _KofN._instances += 1
        self.prefix = f"pdnn_kofn/{os.environ.get('TORCHELASTIC_RESTART_COUNT', '0')}/{_KofN._instances}"
        mk = lambda: dist.TCPStore(host, port, is_master=False, timeout=timedelta(seconds=3600))  # noqa: E731
        self.store, self.wstore = mk(), mk()
        warm_abort_path()
        dist.barrier(group=ddp.pg)                # every rank's clients exist before the first step
        self.abort_step = -1                      # written by the watcher, read by the gradient hooks
        self.done_step = 0
        self.watch_step = 1
        self._stop = False
        self._cv = threading.Condition()
        self._begun = 0
        self._t_begin = {}                        # step -> monotonic begin time (deadline thread)
        self.thread = threading.Thread(target=self._watch, daemon=True)
        self.thread.start()
        if deadline_ms and ddp.rank == 0:         # rank 0 closes a step when its deadline passes
            self.timer = threading.Thread(target=self._deadline, daemon=True)
            self.timer.start()

    def key(self, step, what):
        return f"{self.prefix}/{step}/{what}"

    def begin(self, step):
        with self._cv:
            self._begun = step
            self._t_begin[step] = time.monotonic()
            self._t_begin.pop(step - 8, None)
            self._cv.notify_all()

    def report_done(self, step):
        self.done_step = step
        n = self.store.add(self.key(step, "done"), 1)
        if n == self.k:
            self.store.set(self.key(step, "closed"), "k")

    def _watch(self):
        # blocks server-side on each step's close key in turn (every step is closed: by the k-th finisher,
        # by the deadline, or by stop()) -- no polling traffic
        step = 1
        while not self._stop:
            # a step this rank has already left is over everywhere (its collectives completed): never wait on
            # its key, which cleanup() may already have deleted
            step = max(step, self._begun)
            try:
                self.wstore.wait([self.key(step, "closed")])
            except Exception:
                if self._stop:
                    return
                continue
            if self.done_step < step:             # still computing this step: abandon the rest of it
                self.abort_step = step
            step += 1
            self.watch_step = step

    def _deadline(self):
        # Handles the NEWEST begun step only: steps that began while this thread slept are over (closed by
        # their k-th finisher) or superseded, so it jumps straight to the latest one instead of walking a
        # backlog one deadline at a time, which made a later straggler step's deadline fire late and re-set
        # keys cleanup() had already deleted.
        step = 1
        while not self._stop:
            with self._cv:
                while self._begun < step and not self._stop:
                    self._cv.wait(1.0)
                if self._stop:
                    return
                step = max(step, self._begun)
                t0 = self._t_begin.get(step, time.monotonic())
            try:
                if self.store.check([self.key(step, "closed")]):
                    step += 1                     # already closed by the k-th finisher: no deadline needed
                    continue
            except Exception:
                return
            rest = self.deadline_ms / 1e3 - (time.monotonic() - t0)
            if rest > 0:
                time.sleep(rest)
            try:
                if self._begun == step and not self.store.check([self.key(step, "closed")]):
                    self.store.set(self.key(step, "closed"), "deadline")
            except Exception:
                return
            step += 1

    def cleanup(self, step):
        if self.ddp.rank == 0 and step > 2:
            for w in ("done", "closed"):
                try:
                    self.store.delete_key(self.key(step - 2, w))
                except Exception:
                    pass

    def stop(self):
        self._stop = True
        try:                                      # wake the watcher blocked on the step it is waiting for
            self.store.set(self.key(self.watch_step, "closed"), "stop")
        except Exception:
            pass
        with self._cv:
            self._cv.notify_all()


def warm_abort_path(exc_type=None):
    """Raise and catch one exception from inside an autograd hook.  The FIRST exception that crosses the
    autograd engine costs ~0.3 s of one-time setup on this torch build (0.001 s afterwards): paid here, at
    construction, instead of delaying the first real straggler abort by that much."""
    exc_type = exc_type or StepAborted
    w = torch.ones(1, requires_grad=True)

    def boom(_p):
        raise exc_type("warm-up")
    h = w.register_post_accumulate_grad_hook(boom)
    try:
        (w * 2).sum().backward()
    except exc_type:
        pass
    finally:
        h.remove()


def _work_done(w):
    try:
        return bool(w.is_completed())
    except Exception:
        return False


def _is_nccl(pg):
    try:
        return dist.get_backend(pg) == "nccl"
    except Exception:
        return False


class DistributedDataParallel(nn.Module):
    def __init__(self, module: nn.Module, process_group=None, bucket_cap_mb: float = 32.0,
                 first_bucket_cap_mb: float | None = None, broadcast_buffers: bool = True, comm_dtype=None,
                 average: bool = True, straggler_mode: bool = False, device_ids=None, tracer=None,
                 num_aggregate: int = 0, deadline_ms: float = 0.0, throttle: bool = True,
                 buffer_sync_interval: int = 1, comm_timing: bool = False, split_tied: bool | None = None, last_bucket_cap_mb: float | None = 32.0):
        super().__init__()
        self.module = module
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(process_group) if dist.is_initialized() else 0
        self.flat = flatten_module(module)
        # rank 0's module buffers (BN running statistics) are broadcast every `buffer_sync_interval`
        # training forwards (reference: every forward, data_parallel_dist.py:133-138), so the ranks' BN
        # statistics never drift apart; one collective per dtype over a persistent flat buffer
        self.broadcast_buffers = broadcast_buffers
        self.buffer_sync_interval = max(1, int(buffer_sync_interval))
        self._fwd_count = 0
        self._buf_flat = {}
        # device-side per-bucket all-reduce latency (HIP events, read lazily: no host sync in the step)
        self.comm_timing = comm_timing
        self._ev_log = []
        self._timing_stream = None
        self._ev_bn = None
        self.comm_dtype = comm_dtype
        self.average = average
        self.kofn = None
        self.straggler_mode = straggler_mode or num_aggregate > 0 or deadline_ms > 0
        self.tracer = tracer
        self.throttle = throttle
        self.nccl = _is_nccl(process_group)
        # communicate even at world size 1 (PDNN_DDP_FORCE_COMM=1 with a 1-rank process group): exercises the
        # bucket hooks and RCCL launches on a single GPU exactly as at world size 8
        self._comm = self.world > 1 or (dist.is_initialized() and os.environ.get("PDNN_DDP_FORCE_COMM") == "1")
        self._sync = True
        self.alive = True
        self.grad_scale_dev = None
        self._buffers_list = [b for b in module.buffers() if b is not None and b.numel() > 0]
        self._bn_views = False
        self._bn_work = None             # buffer broadcast issued at the end of the last backward (see forward)
        if self._comm and self.broadcast_buffers:
            self._flatten_bn_buffers()
        if self._comm and self.world > 1 and self.flat.data.is_cuda:
            # RCCL's channel blocks run beside the backward: the persistent GEMM grids leave them CUs
            # (csrc/kernels/tuning.h comm_cus)
            from ..ops import _backend, kernels as K
            if _backend.available():
                K.set_comm_world(self.world)
        self._broadcast_init()
        # split tied embedding (GPT-2's wte = LM head): the head's dense gradient is complete at the START of the
        # backward, the embedding's rows only at its end.  Reduced as one parameter, its 147 MiB bucket could only
        # launch after the embedding backward -- fully exposed at N > 1.  Split: the dense
        # part is bucket 0, all-reduced right after the head's weight gradient; the embedding's B*T rows are
        # gathered (ids + bf16 rows) and added after it (reduce_sparse_rows).  Not with modes that post-process
        # whole buckets (straggler counts, k-of-n, bf16 wire).
        self._tail = None
        early = []
        if split_tied is None:
            split_tied = os.environ.get("PDNN_DDP_SPLIT_TIED", "1") == "1"
        tied = module.ddp_tied_rows() if split_tied and hasattr(module, "ddp_tied_rows") else None
        if (tied is not None and self._comm and not straggler_mode and num_aggregate == 0 and deadline_ms == 0
                and comm_dtype is None):
            early = [tied]
        self._last_cap = last_bucket_cap_mb      # the final bucket's collective is the exposed one (reverse_buckets)
        self._build_buckets(bucket_cap_mb, bucket_cap_mb if first_bucket_cap_mb is None else first_bucket_cap_mb,
                            early)
        if early and self._pbucket.get(id(early[0])) == 0 and self.buckets[0][2] == 1:
            import weakref
            self._tail = early[0]
            module._pdnn_row_tail = weakref.ref(self)
        self._hooks = [register_grad_ready_hook(p, self._on_grad) for p in self.flat.params]
        self.step = 0
        self.last_counts = None          # per-bucket contributor counts of the last step (k-of-n)
        self.aborted_steps = 0
        self._ovl_opt = None           # overlap_optimizer(): per-bucket updates on _ovl_stream
        self._ovl_stream = None
        self._reset()
        self.step_comm_log = []
        self._in_fwd = False
        self.abort_phase = None
        if self._comm and (num_aggregate > 0 or deadline_ms > 0):
            k = num_aggregate if num_aggregate > 0 else self.world
            self.kofn = _KofN(self, min(k, self.world), deadline_ms)
            self._install_forward_checks()

    # ------------------------------------------------------------------ init broadcast (C-13)
    @torch.no_grad()
    def _broadcast_init(self):
        if not self._comm:
            return
        dist.broadcast(self.flat.data, 0, group=self.pg)
        self._broadcast_buffers()
        self.flat.refresh_shadow()

    @torch.no_grad()
    def _flatten_bn_buffers(self):
        """Rebind every BatchNorm buffer as a view of one persistent flat tensor per dtype, so the per-forward
        buffer broadcast is one collective per dtype with no gather/scatter copy kernels (~150 small copies
        per ResNet-50 forward otherwise).  Other buffers keep the copy path."""
        by_dtype, rest = {}, []
        bn_types = (nn.modules.batchnorm._BatchNorm,)
        for mod in self.module.modules():
            for name, b in mod._buffers.items():
                if b is None or b.numel() == 0:
                    continue
                if isinstance(mod, bn_types) and b.is_contiguous():
                    by_dtype.setdefault(b.dtype, []).append((mod, name, b))
                else:
                    rest.append(b)
        for dt, items in by_dtype.items():
            flat = torch.cat([b.reshape(-1) for _, _, b in items])
            o = 0
            for mod, name, b in items:
                n = b.numel()
                mod._buffers[name] = flat[o:o + n].view(b.shape)
                o += n
            self._buf_flat[("bn", dt)] = flat
        self._buffers_list = rest
        self._bn_views = bool(by_dtype)

    @torch.no_grad()
    def _broadcast_buffers(self):
        if not self._comm:
            return
        if self._bn_views:
            for key, flat in self._buf_flat.items():
                if isinstance(key, tuple) and key[0] == "bn":
                    dist.broadcast(flat, 0, group=self.pg)
        if not self._buffers_list:
            return
        by_dtype = {}
        for b in self._buffers_list:
            by_dtype.setdefault(b.dtype, []).append(b)
        for dt, bufs in by_dtype.items():
            n_all = sum(b.numel() for b in bufs)
            flat = self._buf_flat.get(dt)
            if flat is None or flat.numel() != n_all or flat.device != bufs[0].device:
                flat = self._buf_flat[dt] = torch.empty(n_all, dtype=dt, device=bufs[0].device)
            o = 0
            if self.rank == 0:
                for b in bufs:
                    flat[o:o + b.numel()].copy_(b.reshape(-1))
                    o += b.numel()
            dist.broadcast(flat, 0, group=self.pg)
            if self.rank != 0:
                o = 0
                for b in bufs:
                    n = b.numel()
                    b.copy_(flat[o:o + n].view_as(b))
                    o += n

    # ------------------------------------------------------------------ buckets
    def _build_buckets(self, cap_mb, first_mb, early=()):
        self.buckets, self._pbucket = reverse_buckets(self.flat, cap_mb, first_mb, early,
                                                      getattr(self, "_last_cap", None))
        if self.comm_dtype is not None:
            self._wire = [torch.empty(e - s, dtype=self.comm_dtype, device=self.flat.grad.device) for s, e, _ in self.buckets]

    def bucket_sizes_mb(self):
        return [(e - s) * 4 / 2 ** 20 for s, e, _ in self.buckets]

    # ------------------------------------------------------------------ forward-phase short-circuit
    def _install_forward_checks(self):
        """k-of-n: a rank whose step is closed while it is still in its FORWARD abandons the step before its
        next layer (the C++ worker checks before every forward layer too, worker_nn.h:56-64; the reference's
        PyTorch worker polls the kill tag before each layer, lenet.py:168-178).  Checked at every parameter's
        use through ``p._pdnn_await``: the fused GPU ops call it when they fetch a weight's bf16 shadow, and
        :class:`~..optim.flat.ParamUseMode` around the forward calls it for torch ops taking a parameter."""
        for p in self.flat.params:
            if "_pdnn_await" not in p.__dict__:
                p._pdnn_await = lambda _p: self._forward_check()

    def _forward_check(self):
        # during the forward of step self.step + 1 the watcher flags that step once it is closed elsewhere
        if self._in_fwd and self.kofn is not None and self.kofn.abort_step == self.step + 1:
            self._in_fwd = False
            raise StepAborted(f"rank {self.rank} step {self.step + 1} (forward)")

    def _abort_forward(self):
        """The step was closed during this rank's forward: no backward runs, so take part in the step's
        collectives here -- every bucket zero-filled, then the contributor counts -- exactly as an abort in the
        backward would (_finish), leaving the count-correct average in the gradient arena."""
        self._reset()
        self._armed = True
        self.step += 1
        self._t0 = time.perf_counter()
        self.kofn.begin(self.step)
        self._aborted = True
        self.abort_phase = "forward"
        self._finish()

    # ------------------------------------------------------------------ per-backward state
    def _reset(self):
        self._ready = [0] * len(self.buckets)
        self._next = 0
        self._works = []
        self._work_of = {}
        self._tail_pending = None
        self._armed = False
        self._aborted = False
        self._contrib = [0.0] * len(self.buckets)
        self._events = []
        self.launch_order = []
        self._ev_start, self._ev_done = {}, {}
        self._ovl_step = False          # this step's buckets are being applied by the overlapped optimizer

    def _arm(self):
        self.abort_phase = None
        self._armed = True
        self.step += 1
        self._t0 = time.perf_counter()
        if self.comm_timing and self.flat.grad.is_cuda:
            self._ev_arm = torch.cuda.Event(enable_timing=True)
            self._ev_arm.record()
        torch.autograd.Variable._execution_engine.queue_callback(self._finish)
        if self.kofn is not None:
            self.kofn.begin(self.step)

    def _on_grad(self, p):  # noqa: D401 - side-aware grad-ready hook (see _launch)
        if not self._sync or not self._comm or self._aborted:
            return
        if not self._armed:
            self._arm()
        if self.kofn is not None and self.kofn.abort_step == self.step:
            self._aborted = True                 # closed by the k-th finisher / deadline: short-circuit
            self.abort_phase = "backward"
            raise StepAborted(f"rank {self.rank} step {self.step}")
        b = self._pbucket[id(p)]
        self._ready[b] += 1
        while self._next < len(self.buckets) and self._ready[self._next] == self.buckets[self._next][2]:
            self._launch(self._next)
            self._next += 1
        if self.kofn is not None and self._next == len(self.buckets):
            self.kofn.report_done(self.step)     # this rank's full gradient is in flight

    def _op(self):
        if self.straggler_mode or not self.average:
            return dist.ReduceOp.SUM
        # one rank: the average IS the sum, and RCCL runs an in-place one-rank SUM as a no-op, where AVG launched
        # a scale-by-1 pass over every bucket (0.42 ms of HBM traffic per ResNet-50 step, BENCH_r04 comm block)
        return dist.ReduceOp.AVG if self.nccl and self.world > 1 else dist.ReduceOp.SUM

    def _launch(self, b, zero=False):
        # Fused ResNet blocks write weight gradients on a side stream and do not join it back before announcing
        # them (ops/fused_resnet.py): the bucket's collective (and any zero-fill / cast of the bucket) is issued
        # from the side stream after it has caught up with the compute stream, so it is ordered after both
        # while the compute stream runs on into the next block's backward.
        if self.kofn is not None and self.throttle and self.flat.grad.is_cuda:
            # keep the host at most two buckets ahead of the GPU, so an abort stops real GPU work.  The event is
            # recorded on the COMPUTE stream (the data-gradient chain): recorded on the weight-gradient side
            # stream, which runs at low priority and lags, it held the host back until the side stream caught up
            # and starved the compute stream (k-of-n at world 1: 8,371 vs 9,409 img/s, gpurun_out/r3_09)
            if len(self._events) >= 2:
                self._events[-2].synchronize()
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.flat.grad.device))
            self._events.append(ev)
        side = side_stream_if_active(self.flat.grad)
        if side is None:
            return self._launch_on(b, zero)
        from ..ops import kernels as K
        K.stream_wait(side, torch.cuda.current_stream(side.device))
        with torch.cuda.stream(side):
            return self._launch_on(b, zero)

    def _launch_on(self, b, zero=False):
        s, e, _ = self.buckets[b]
        view = self.flat.grad[s:e]
        if self.straggler_mode and (zero or not self.alive):
            view.zero_()                       # zero contribution: collective stays matched
        else:
            self._contrib[b] = 1.0
        t = view
        if self.comm_dtype is not None:
            t = self._wire[b]
            scale = 1.0 / self.world if (self.average and not self.straggler_mode) else 1.0
            if view.is_cuda:
                from ..ops import kernels as K
                K.cast_f32_bf16(view, t, scale) if t.dtype == torch.bfloat16 else t.copy_(view * scale)
            else:
                t.copy_(view * scale)
            op = dist.ReduceOp.SUM
        else:
            op = self._op()
        if self.tracer is not None:
            self.tracer.instant(f"allreduce_bucket{b}", args={"mb": (e - s) * 4 / 2 ** 20})
        self.launch_order.append(b)
        if self.comm_timing and view.is_cuda and getattr(self, "_ev_arm", None) is not None:
            # the collective issued from a timing stream that has nothing else queued: its start event fires when
            # the bucket's gradients are ready (the stream waits on the launching one), its end event when RCCL's
            # kernel is done (the stream waits on RCCL's) -- per-bucket device time, no host sync in the step
            if self._timing_stream is None:
                self._timing_stream = torch.cuda.Stream(device=view.device)
            cs = self._timing_stream
            cs.wait_stream(torch.cuda.current_stream(view.device))
            with torch.cuda.stream(cs):
                ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                ev0.record(cs)
                work = dist.all_reduce(t, op=op, group=self.pg, async_op=True)
                work.wait()
                ev1.record(cs)
            t.record_stream(cs)
            self._ev_start[b], self._ev_done[b] = ev0, ev1
            self._works.append((b, work))
            self._work_of[b] = work
            return
        work = dist.all_reduce(t, op=op, group=self.pg, async_op=True)
        self._works.append((b, work))
        self._work_of[b] = work
        if self._ovl_active():
            # the bucket's optimizer update on the optimizer stream, as soon as its all-reduce is done, beside
            # the backward of the earlier layers (whose weights it does not touch)
            opt = self._ovl_opt
            if not self._ovl_step:
                opt._overlap_begin()           # host side: step counter / state, before the first range
                self._ovl_step = True
            os_ = self._ovl_stream
            with torch.cuda.stream(os_):
                work.wait()                    # the optimizer stream waits for RCCL's
                opt._overlap_range(s, e)

    def _ovl_active(self):
        return (self._ovl_opt is not None and self.comm_dtype is None and not self.straggler_mode
                and self.kofn is None and not self.comm_timing and not self._aborted and self.flat.grad.is_cuda
                and not self._ovl_opt._graph and self._ovl_reduced_is_final())

    def _ovl_reduced_is_final(self):
        """Whether a bucket is final the moment its collective completes: RCCL reduces with native AVG, and a
        SUM is final when no average is wanted or there is one rank.  Over gloo (SUM, then ``grad *= 1/world``
        in _finish after every wait) a per-bucket update would consume world x the averaged gradient,
        so the overlap stays off there and opt.step() runs after the backward as usual."""
        return self.nccl or not self.average or self.world == 1

    def overlap_optimizer(self, opt):
        """Apply ``opt``'s update bucket by bucket during the backward: each bucket's range of the flat arena is
        updated on an optimizer stream right after its all-reduce, while the compute stream runs the backward of
        the earlier layers; ``opt.step()`` after the backward then has nothing left to do (it still works as usual
        for a step without buckets, e.g. under ``no_sync``).  ``opt`` must be a fused flat optimizer whose single
        param group spans exactly this wrapper's buckets.  Returns ``opt``; None (no overlap) when it does not
        qualify.

        The updates run DURING the backward: the hyper-parameters (lr, momentum, weight decay) are read when the
        step's first bucket launches, and nothing that runs between ``backward()`` and ``opt.step()`` (gradient
        clipping, manual gradient edits, lr changes) reaches them -- Trainer refuses ``grad_clip`` with it."""
        ok = opt._overlap_ok() if hasattr(opt, "_overlap_ok") else None
        if ok is None or ok[0] is not self.flat or self._tail is not None:
            # (a split tied embedding gets its sparse rows after its bucket's collective: not final there)
            return None
        s, e = ok[1]
        ranges = sorted((bs, be) for bs, be, _ in self.buckets)
        if not ranges or ranges[0][0] != s or ranges[-1][1] != e or any(ranges[i][1] != ranges[i + 1][0]
                                                                         for i in range(len(ranges) - 1)):
            return None
        self._ovl_opt = opt
        self._ovl_stream = torch.cuda.Stream(device=self.flat.grad.device)
        return opt

    def _finish(self):
        if not self._armed:
            return
        while self._next < len(self.buckets):      # unused parameters, or everything after an abort
            self._launch(self._next, zero=self._aborted)
            self._next += 1
        if self.kofn is not None and not self._aborted and self.kofn.done_step < self.step:
            # buckets of parameters without a gradient launch only here: this rank's gradient is now complete
            # (otherwise no rank reports and the k-th-finisher close never fires)
            self.kofn.report_done(self.step)
        fp = self.flat
        ev_bwd = None
        if self.comm_timing and fp.grad.is_cuda and getattr(self, "_ev_arm", None) is not None:
            # the backward's last kernels: compute stream, and the weight-gradient side stream if active
            ev_bwd = [torch.cuda.Event(enable_timing=True)]
            ev_bwd[0].record()
            side = side_stream_if_active(fp.grad)
            if side is not None:
                ev_bwd.append(torch.cuda.Event(enable_timing=True))
                ev_bwd[1].record(side)
        if self.straggler_mode:
            # per-bucket contributor counts: all-reduced after the buckets (same collective order everywhere)
            # staged through pinned host memory: a pageable host->device copy would block the host until the
            # whole backward has run (a full sync per step: k-of-n 25.10 vs DDP 23.95 ms, gpurun_out/r4_09)
            cnt = torch.tensor(self._contrib, dtype=torch.float32, pin_memory=fp.grad.is_cuda)
            cnt = cnt.to(fp.grad.device, non_blocking=True)
            self._works.append((-1, dist.all_reduce(cnt, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)))
        self._issue_buffer_broadcast()
        for b, w in self._works:
            w.wait()
        if self._ovl_step:
            # every bucket's update was queued on the optimizer stream: the compute stream (the next zero_grad /
            # forward) waits for them, and the optimizer's step() finds them applied
            torch.cuda.current_stream(fp.grad.device).wait_stream(self._ovl_stream)
            self._ovl_opt._overlap_end()
        if ev_bwd is not None and self._ev_start:
            self._ev_log.append({"arm": self._ev_arm, "bwd": ev_bwd, "bn": self._ev_bn,
                                 "buckets": [(b, self._ev_start[b], self._ev_done[b]) for b in sorted(self._ev_start)]})
        self._ev_arm = self._ev_bn = None
        if self.comm_dtype is not None:
            for b, (s, e, _) in enumerate(self.buckets):
                fp.grad[s:e].copy_(self._wire[b])
        elif self.average and not self.straggler_mode and not self.nccl:
            fp.grad.mul_(1.0 / self.world)
        if self.straggler_mode:
            # every bucket divided by ITS count (device tensors: no host sync on GPU)
            inv = torch.reciprocal(cnt.clamp_min(1.0))
            for b, (s, e, _) in enumerate(self.buckets):
                fp.grad[s:e].mul_(inv[b])
            self.last_counts = cnt
            self.grad_scale_dev = None
            for opt in getattr(self, "_optimizers", []):
                opt.grad_scale_dev = None
        if self._tail_pending is not None:        # split tied embedding: its gathered rows on top of the average
            idx, rows, apply = self._tail_pending
            self._tail_pending = None
            apply(idx, rows, 1.0 / self.world if self.average else 1.0)
        if self.kofn is not None:
            self.kofn.cleanup(self.step)
        self.last_contrib = list(self._contrib)
        self.last_launch_order = list(self.launch_order)
        self.aborted_steps += int(self._aborted)
        self.step_comm_log.append(time.perf_counter() - self._t0)
        self._reset()

    # ------------------------------------------------------------------ split tied embedding
    def reduce_sparse_rows(self, p, idx, rows, apply):
        """The embedding part of a split tied parameter (``self._tail``, see __init__): ``rows[m]`` is this rank's
        gradient for row ``idx[m]`` of ``p`` (every rank passes the same number of rows).  The rows and ids of every
        rank are all-gathered (bf16 rows stay bf16 on the wire: ~12.6 MB per rank for GPT-2 at B*T = 8192) and
        ``apply(idx_all, rows_all, scale)`` adds them into p's gradient at the end of the backward (_finish), after
        every bucket's collective has completed and the arena holds its final average (or the bf16 wire copy):
        scale = 1/world when averaging.  Outside a synchronised step (no_sync) the local rows are added as they
        are, at once."""
        idx = idx.reshape(-1).contiguous()
        rows = rows.reshape(idx.numel(), -1).contiguous()
        if not (self._sync and self._comm) or self._aborted or p is not self._tail:
            apply(idx, rows, 1.0)
            return
        if self._work_of.get(self._pbucket[id(p)]) is None:
            raise RuntimeError("reduce_sparse_rows: the dense part of the split tied parameter was not announced "
                               "(its grad-ready hook must fire before the embedding backward)")
        if self.world > 1:
            ia = torch.empty(self.world * idx.numel(), dtype=idx.dtype, device=idx.device)
            ra = torch.empty((self.world * rows.shape[0], rows.shape[1]), dtype=rows.dtype, device=rows.device)
            dist.all_gather_into_tensor(ia, idx, group=self.pg)
            dist.all_gather_into_tensor(ra, rows, group=self.pg)
            idx, rows = ia, ra
        self._tail_pending = (idx, rows, apply)

    # ------------------------------------------------------------------ public API
    def backward(self, loss):
        """``loss.backward()`` that tolerates a k-of-n abort: the rest of the backward is skipped, the
        remaining buckets are all-reduced zero-filled and the step completes with count-correct buckets.
        Returns True when this rank was short-circuited."""
        try:
            loss.backward()
            return False
        except StepAborted:
            self._finish()
            return True

    def close(self):
        if self.kofn is not None:
            self.kofn.stop()

    def _buffer_sync_due(self):
        return (self.broadcast_buffers and self._comm and self.module.training
                and self._fwd_count % self.buffer_sync_interval == 0)

    @torch.no_grad()
    def _issue_buffer_broadcast(self):
        """End of a backward: broadcast rank 0's BatchNorm buffers for the NEXT training forward now, behind the
        last gradient bucket on the communicator's stream.  Only the forward changes the buffers, so their
        values here equal those at the next forward's start (where the reference broadcasts them,
        data_parallel_dist.py:133-138); issued here, the collective overlaps the optimizer step instead of
        being a cross-rank sync point in front of the forward's first kernel, and forward() only makes its
        stream wait for it (a device-side wait on RCCL).  The int64 step counters and any non-BN buffers keep
        the forward-time path."""
        self._bn_work = None
        if not (self._bn_views and self._buffer_sync_due()) or self._buffers_list:
            return
        flats = [flat for key, flat in self._buf_flat.items() if isinstance(key, tuple) and key[0] == "bn"]
        side = side_stream_if_active(self.flat.grad)
        if side is not None:
            # issued from the weight-gradient side stream after a fence-free wait, like the bucket collectives
            # (_launch), so the collective's event record lands off the compute stream
            from ..ops import kernels as K
            K.stream_wait(side, torch.cuda.current_stream(side.device))
            with torch.cuda.stream(side):
                works = [dist.broadcast(flat, 0, group=self.pg, async_op=True) for flat in flats]
        else:
            works = [dist.broadcast(flat, 0, group=self.pg, async_op=True) for flat in flats]
        self._bn_work = (works, self._fwd_count)

    def forward(self, *args, **kwargs):
        """Raises :class:`StepAborted` when k-of-n closed this step during the forward (after the step's
        collectives have completed with a zero contribution from this rank): skip the loss and backward and
        go on to the optimizer step, as after ``backward(loss)`` returned True."""
        if self.broadcast_buffers and self._comm and self.module.training:
            if self._fwd_count % self.buffer_sync_interval == 0:
                pre = self._bn_work
                self._bn_work = None
                if pre is not None and pre[1] == self._fwd_count:
                    # issued after the last backward: the stream waits, the host does not.  Timed: the compute
                    # stream's stall on it (0 when it finished during the optimizer step)
                    timed = self.comm_timing and self.flat.grad.is_cuda
                    if timed:
                        self._ev_bn = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                        self._ev_bn[0].record()
                    for w in pre[0]:
                        w.wait()
                    if timed:
                        self._ev_bn[1].record()
                elif self.comm_timing and self.flat.grad.is_cuda:
                    self._ev_bn = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                    self._ev_bn[0].record()
                    self._broadcast_buffers()
                    self._ev_bn[1].record()
                else:
                    self._broadcast_buffers()
            self._fwd_count += 1
        if self.kofn is None or not (self.module.training and self._sync and torch.is_grad_enabled()):
            return self.module(*args, **kwargs)
        self._in_fwd = True
        awaits = getattr(self.module, "awaits_params", None)
        mode = (contextlib.nullcontext() if awaits is not None and awaits(*args, **kwargs)
                else ParamUseMode(lambda: self.kofn.abort_step == self.step + 1))
        try:
            with mode:
                return self.module(*args, **kwargs)
        except StepAborted:
            self._abort_forward()
            raise
        finally:
            self._in_fwd = False

    def progress(self):
        """Where this rank's gradient communication stands, without blocking (a hang watchdog reads it from its
        own thread): the step being reduced, the buckets launched so far in it, and the last bucket whose
        collective has completed (``Work.is_completed`` is a query, not a wait)."""
        works = list(self._works)
        done = [b for b, w in works if b >= 0 and _work_done(w)]
        return {"step": self.step, "in_backward": self._armed, "buckets": len(self.buckets),
                "last_bucket_launched": self.launch_order[-1] if self.launch_order else None,
                "last_bucket_completed": max(done) if done else None,
                "buckets_in_flight": [b for b, w in works if b >= 0 and b not in done]}

    def sync_buffers(self):
        """Broadcast rank 0's buffers now (e.g. before evaluation or a checkpoint: the last training forward
        updated every rank's BN running statistics with its own batch)."""
        self._broadcast_buffers()

    def comm_times_ms(self):
        """Per step, per bucket: device time of the bucket's all-reduce, from its gradients being ready to
        RCCL's kernel completing (``comm_timing=True``), for the steps logged since the last call.  Synchronises
        on the recorded events."""
        return [r["bucket_ms"] for r in self.comm_records()]

    def comm_records(self):
        """Per logged step (``comm_timing=True``): ``bucket_ms`` (per bucket, ready -> all-reduced),
        ``bucket_ready_ms`` / ``bucket_done_ms`` (from the first gradient hook), ``bwd_end_ms`` (last backward
        kernel, both streams), ``tail_ms`` (last bucket done minus the backward's end: the exposed
        communication) and ``bn_bcast_ms`` (what the BatchNorm-buffer broadcast cost the forward's stream: the
        whole collective when issued at the forward, the stall on it when it was issued after the previous
        backward).  Synchronises."""
        out = []
        for r in self._ev_log:
            arm = r["arm"]
            arm.synchronize()
            ready = [arm.elapsed_time(s) for _, s, _ in r["buckets"]]
            done = [arm.elapsed_time(e) for _, _, e in r["buckets"]]
            bwd = max(arm.elapsed_time(e) for e in r["bwd"])
            rec = {"bucket_ms": [d - s for s, d in zip(ready, done)], "bucket_ready_ms": ready,
                   "bucket_done_ms": done, "bwd_end_ms": bwd, "tail_ms": max(0.0, max(done) - bwd),
                   "bn_bcast_ms": r["bn"][0].elapsed_time(r["bn"][1]) if r["bn"] is not None else None}
            out.append(rec)
        self._ev_log = []
        return out

    def set_comm_dtype(self, dtype):
        """Switch the wire dtype between steps (None = the fp32 gradients themselves, torch.bfloat16 = a cast
        copy per bucket)."""
        self.comm_dtype = dtype
        if dtype is not None:
            self._wire = [torch.empty(e - s, dtype=dtype, device=self.flat.grad.device) for s, e, _ in self.buckets]

    @contextlib.contextmanager
    def no_sync(self):
        old = self._sync
        self._sync = False
        try:
            yield
        finally:
            self._sync = old

    def set_alive(self, alive: bool):
        """Straggler mode: this rank's gradient contributes (True) or is dropped this step (False)."""
        self.alive = bool(alive)

    def attach_optimizer(self, opt):
        """Let the fused optimizer consume the device-side 1/alive scale in straggler mode."""
        self._optimizers = getattr(self, "_optimizers", []) + [opt]
        return opt

    def zero_grad(self):
        self.flat.zero_grad()

    def state_dict(self, *a, **kw):   # "module."-prefixed keys like torch DDP (data_parallel_dist.py:38)
        return super().state_dict(*a, **kw)


DistributedDataParallel._on_grad._pdnn_side_aware = True
