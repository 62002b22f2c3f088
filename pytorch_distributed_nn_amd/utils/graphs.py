"""hipGraph-captured training step: forward + loss + backward + fused optimizer replayed as ONE graph.

Why (MI355X-first): a training step of this framework is a few hundred to ~2000 small kernel launches
issued from Python through ctypes.  For the reference's own configurations (LeNet / CIFAR ResNets at
batch 128: pytorch_code/distributed_nn.py:42, single_machine.py:184-205) the GPU work per kernel is
microseconds, so an eager step is bound by host launch cost, not by the GPU.  A captured hipGraph
(``torch.cuda.CUDAGraph`` is hipGraph on ROCm) replays the whole step with one host call.  The reference
has no counterpart (its CPU loop is pytorch_code/nn_ops/__init__.py:46-85); this is the MI355X answer to
"capture launch-bound inner loops in hipGraphs".

How it stays correct:

* every kernel of the framework is launched on ``torch.cuda.current_stream()`` (``ops/_backend.py``),
  so capture records them in order; no op syncs with the host inside a step;
* activations/workspaces allocated during capture come from the graph's private memory pool and are
  reused by every replay;
* inputs are copied into static tensors before each replay;
* the fused optimizers switch to **graph mode** (``optim.fused``): the per-step values that a graph
  would otherwise freeze (learning rate of a schedule, Adam's bias corrections) are read by the kernel
  from a device buffer that :meth:`~..optim.fused._FusedBase.pre_replay` refreshes with stream-ordered
  fills before every replay;
* the first ``warmup`` calls run eagerly (lazy workspace allocation, fp8 amax priming, momentum-buffer
  initialisation happen there), the next call captures and replays.

Batches whose shapes differ from the captured ones (e.g. a final partial batch) run eagerly.  A DDP
model with world size > 1 would capture its RCCL all-reduces too; that is opt-in
(``allow_collectives=True``) because every rank must then capture the identical collective sequence.
"""
from __future__ import annotations

import torch


class GraphedStep:
    """``step = GraphedStep(model, opt, loss_fn); loss = step(x, y)`` — one training iteration per call.

    ``forward(model, x, y) -> loss`` overrides the default ``loss_fn(model(x), y)`` (e.g. language models
    that compute their loss internally).  The returned loss / :attr:`output` tensors are static: they are
    overwritten by the next call, read them (or ``.clone()``) before calling again.
    """

    def __init__(self, model, optimizer, loss_fn=None, forward=None, warmup: int = 2, enabled: bool | None = None,
                 allow_collectives: bool = False, grad_clip: float | None = None):
        self.model, self.opt = model, optimizer
        self.loss_fn = loss_fn
        self._forward = forward
        self.grad_clip = grad_clip
        self.warmup = max(1, int(warmup))
        self.enabled = enabled
        self.allow_collectives = allow_collectives
        self.graph = None
        self.static_x = self.static_y = None
        self.static_loss = None
        self.output = None
        self.eager_calls = 0
        self.replays = 0

    # ------------------------------------------------------------------------------------------------
    def _fwd(self, x, y):
        if self._forward is not None:
            return self._forward(self.model, x, y), None
        out = self.model(x)
        return self.loss_fn(out, y), out

    def _eager(self, x, y):
        self.opt.zero_grad()
        loss, out = self._fwd(x, y)
        loss.backward()
        if self.grad_clip:           # device-side norm + clamp: no host sync, capturable
            torch.nn.utils.clip_grad_norm_(self.model.parameters(), self.grad_clip, foreach=True)
        self.opt.step()
        # Only DETACHED results leave a step: a live autograd graph from an eager step (held by a returned
        # loss/logits) keeps the parameters' AccumulateGrad nodes, created on the eager stream, alive into
        # the capture, where they would sync with that stream and break it (HIP crashes in capture_end).
        return loss.detach(), (out.detach() if out is not None else None)

    def _check_collectives(self):
        world = getattr(self.model, "world", 1)
        if world > 1 and not self.allow_collectives:
            raise RuntimeError("GraphedStep: the model all-reduces across ranks; pass allow_collectives=True "
                               "to capture the RCCL collectives into the graph")

    def _capture(self, x, y):
        self._check_collectives()
        self.static_x = x.detach().clone()
        self.static_y = y.detach().clone()
        torch.cuda.synchronize()
        self.opt.graph_mode(True)
        self.graph = torch.cuda.CUDAGraph()
        # thread_local: a data-loader thread doing its own H2D copies must not invalidate the capture
        with torch.cuda.graph(self.graph, capture_error_mode="thread_local"):
            self.static_loss, self.output = self._fwd_bwd_step_static()

    def _fwd_bwd_step_static(self):
        return self._eager(self.static_x, self.static_y)

    def _same_shape(self, x, y):
        return (x.shape == self.static_x.shape and y.shape == self.static_y.shape and x.dtype == self.static_x.dtype
                and y.dtype == self.static_y.dtype)

    # ------------------------------------------------------------------------------------------------
    def __call__(self, x, y):
        enabled = x.is_cuda if self.enabled is None else self.enabled
        if not enabled:
            return self._eager(x, y)[0]
        if self.graph is None:
            if self.eager_calls < self.warmup:
                self.eager_calls += 1
                loss, self.output = self._eager(x, y)
                return loss
            self._capture(x, y)
        elif not self._same_shape(x, y):
            self.opt.graph_mode(False)
            try:
                loss, self.output = self._eager(x, y)
            finally:
                self.opt.graph_mode(True)
            return loss
        if x.data_ptr() != self.static_x.data_ptr():
            self.static_x.copy_(x, non_blocking=True)
        if y.data_ptr() != self.static_y.data_ptr():
            self.static_y.copy_(y, non_blocking=True)
        self.opt.pre_replay()
        self.graph.replay()
        self.replays += 1
        # the replayed optimizer updated the flat arenas without running host code: bump their update
        # generation so host-side caches keyed on it (transposed / fp8 weight copies) rebuild when an
        # eager call follows (inside the graph they are rebuilt by captured kernels on every replay)
        for fp in self._flat_arenas():
            fp.generation += 1
        return self.static_loss

    def _flat_arenas(self):
        if not hasattr(self, "_flats"):
            seen = {}
            for p in self.model.parameters():
                fp = getattr(p, "_pdnn_flat", None)
                if fp is not None:
                    seen[id(fp)] = fp
            self._flats = list(seen.values())
        return self._flats

    def reset(self):
        """Drop the captured graph (e.g. after changing the model); the next call re-captures."""
        if self.graph is not None:
            self.opt.graph_mode(False)
        self.graph = None
        self.eager_calls = self.warmup
