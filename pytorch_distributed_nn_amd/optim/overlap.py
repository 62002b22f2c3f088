"""Optimizer step overlapped with the backward (single process, fused Adam/AdamW on a flat arena).

The fused optimizers (``optim/fused.py``) update the whole flat arena in one launch after the backward; for
GPT-2 small that launch streams ~3.7 GB (fp32 weights, gradients, two moments, bf16 shadow: 30 B per
parameter) while the GPU does nothing else.  Here the arena is cut into reverse-order chunks
(``reverse_buckets``, the same grouping the DDP buckets use) and each chunk is updated on a side HIP stream
as soon as the grad-ready hooks report all of its parameters complete, so the memory-bound optimizer runs
under the remaining (GEMM-bound) backward instead of after it.  The reference has no counterpart (its
optimizers run after ``backward()``: pytorch_code/optim/sgd.py, distributed_TF/src/distributed_train.py).

Correctness: a chunk's kernel is ordered after everything queued on the compute stream when its last
parameter reported (its gradient producers); parameters are only read by the backward of the layers that
own them, which precedes their readiness (tied weights -- GPT-2's wte -- report once, after their last use,
in the embedding backward); the compute stream joins the side stream at the end of the backward, before
the next forward reads the weights or their bf16 shadow.  Gradient clipping needs every gradient first and
is therefore not supported in this mode.

Measured on GPT-2 small bs8 (one MI355X, gpurun_out/r2_41): 464k tokens/s overlapped vs 464-465k eager and
467-469k graphed whole-arena steps -- the persistent ping-pong GEMM kernels hold every CU through the
backward, so the chunks find no idle bandwidth to fill.  Opt-in (``bench.py``: PDNN_OPT_OVERLAP=1).
"""
from __future__ import annotations

import torch

from .flat import register_grad_ready_hook, reverse_buckets
from .fused import Adam


class BackwardOverlappedStep:
    """``ov = BackwardOverlappedStep(opt); opt.zero_grad(); ov.arm(); loss.backward()`` — the step happens
    during the backward (``opt.step()`` must not be called as well)."""

    def __init__(self, opt, chunk_mb: float = 32.0, first_mb: float = 8.0):
        if len(opt.param_groups) != 1:
            raise ValueError("BackwardOverlappedStep: one param group covering the flat arena")
        self.opt = opt
        fp, rng = opt._group_flat(0, opt.param_groups[0])
        if fp is None or rng != (0, fp.numel) or not fp.data.is_cuda:
            raise ValueError("BackwardOverlappedStep: the group must cover a whole CUDA flat arena")
        self.fp = fp
        if not isinstance(opt, Adam):
            raise TypeError("BackwardOverlappedStep: fused Adam / AdamW only")
        self.chunks, self._pchunk = reverse_buckets(fp, chunk_mb, first_mb)
        self.side = torch.cuda.Stream(device=fp.data.device)
        self._hooks = [register_grad_ready_hook(p, self._on_grad) for p in fp.params]
        self._armed = False
        self.steps = 0

    def close(self):
        for h in self._hooks:
            h.remove()

    # ------------------------------------------------------------------------------------------------
    def arm(self):
        """Call after zero_grad and before backward: the next backward performs the optimizer step."""
        g = self.opt.param_groups[0]
        st = self.opt.state.setdefault("flat0", {})
        n = self.fp.numel
        dev = self.fp.data.device
        if "step" not in st:
            st["step"] = 0
            st["exp_avg"] = torch.zeros(n, device=dev)
            st["exp_avg_sq"] = torch.zeros(n, device=dev)
        st["step"] += 1
        t = st["step"]
        b1, b2 = g["betas"]
        self._args = (g["lr"], b1, b2, g["eps"], g["weight_decay"], self.opt.decoupled, 1 - b1 ** t, 1 - b2 ** t)
        self._ready = [0] * len(self.chunks)
        self._done = [False] * len(self.chunks)
        self._armed = True
        self._queued = False

    def _on_grad(self, p):
        if not self._armed:
            return
        if not self._queued:
            self._queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self._finish)
        b = self._pchunk[id(p)]
        self._ready[b] += 1
        if self._ready[b] == self.chunks[b][2]:
            self._launch(b)

    def _launch(self, b):
        if self._done[b]:
            return
        self._done[b] = True
        s, e, _ = self.chunks[b]
        self.side.wait_stream(torch.cuda.current_stream(self.side.device))
        with torch.cuda.stream(self.side):
            self._update(s, e)

    def _update(self, s, e):
        from ..ops import kernels as K
        fp, st = self.fp, self.opt.state["flat0"]
        sh = fp.shadow[s:e] if fp.shadow is not None else None
        lr, b1, b2, eps, wd, dec, bc1, bc2 = self._args
        K.adam_step(fp.data[s:e], fp.grad[s:e], st["exp_avg"][s:e], st["exp_avg_sq"][s:e], sh, lr, b1, b2, eps, wd,
                    dec, bc1, bc2, self.opt.grad_scale_dev, self.opt.grad_scale)

    def _finish(self):
        for b in range(len(self.chunks)):        # chunks whose parameters got no gradient this backward
            if not self._done[b]:
                self._launch(b)
        torch.cuda.current_stream(self.side.device).wait_stream(self.side)
        self.fp.generation += 1
        self._armed = False
        self.steps += 1
