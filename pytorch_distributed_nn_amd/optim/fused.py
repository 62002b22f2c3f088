"""Fused flat-buffer optimizers: SGD (momentum / dampening / weight decay / Nesterov) and Adam / AdamW.

torch.optim-compatible API (``param_groups``, ``zero_grad``, ``state_dict``/``load_state_dict``,
``step(closure)``), semantics identical to ``torch.optim.SGD`` / ``Adam`` / ``AdamW``.

When a param group covers a contiguous range of a :class:`~.flat.FlatParams` arena (the normal case:
``SGD(model.parameters())`` after ``flatten_module``/DDP) the whole group is ONE kernel launch
(``optim.hip``) that also refreshes the bf16 weight shadow and applies the gradient averaging factor
(``grad_scale``, or a device-side scale such as 1/alive-count for the straggler-tolerant modes).  Groups
that are not flat fall back to one launch per tensor (GPU) or the torch reference update (CPU).

Reference parity: the PS master applies ``param -= lr * avg_grad`` (sync_replicas_master_nn.py:22-28,
216-219) and ignores --momentum (defect D9); the C++ master fuses the average into the update as
``ApplyGrad(lr / count)`` (sync_replicas_master_nn.h:124-128); the TF stack uses Adam
(distributed_train.py:160).  Here momentum IS honoured and the average is fused the C++ way.
"""
from __future__ import annotations

import math

import torch

from .flat import FlatParams


def _flat_of(params):
    fps = {id(getattr(p, "_pdnn_flat", None)) for p in params}
    if len(fps) != 1:
        return None, None
    fp = getattr(params[0], "_pdnn_flat", None)
    if fp is None:
        return None, None
    rng = fp.param_range(params)
    return (fp, rng) if rng is not None else (None, None)


class _FusedBase(torch.optim.Optimizer):
    def __init__(self, params, defaults):
        super().__init__(params, defaults)
        self.grad_scale = 1.0          # host-side factor (e.g. 1/world_size when grads are summed)
        self.grad_scale_dev = None     # optional device scalar (e.g. 1/alive for k-of-n)
        self._flat_cache = {}
        self._graph = False            # graph mode: per-step hyper-parameters live in device memory
        self._hyper = {}

    def _group_flat(self, gi, group):
        if gi not in self._flat_cache:
            self._flat_cache[gi] = _flat_of(group["params"])
        return self._flat_cache[gi]

    # ---------------------------------------------------------------------------------- graph mode
    # A hipGraph captured around ``step()`` replays the kernels with the arguments they had at capture.
    # In graph mode the fused kernels read the values that change between steps (lr; Adam's bias
    # corrections) from a per-group device buffer instead, and :meth:`pre_replay` — called on the host
    # before every replay — advances the host-side state and refreshes that buffer with stream-ordered
    # fills (no host<->device sync, so the CPU can run ahead of the GPU as in eager mode).
    _HYPER_LEN = 1

    def graph_mode(self, on: bool = True):
        if on:
            for gi, group in enumerate(self.param_groups):
                fp, _ = self._group_flat(gi, group)
                if fp is None or not fp.data.is_cuda:
                    raise RuntimeError("graph mode needs every param group on a flat CUDA arena")
                self._check_graphable(gi)
                # allocated (and filled) OUTSIDE any capture: a buffer created inside the capture would
                # come from the graph pool and its initialising fill would be replayed over pre_replay's
                if gi not in self._hyper:
                    self._hyper[gi] = torch.zeros(self._HYPER_LEN, dtype=torch.float32, device=fp.data.device)
                    self._fill_hyper(gi, group, advance=False)
        self._graph = bool(on)

    def _check_graphable(self, gi):
        pass

    def _hyper_buf(self, gi, n, device):
        return self._hyper[gi]

    def _hyper_values(self, gi, group, advance=True):    # one step's values, in the kernel's hyper[] order
        return [group["lr"]]

    @torch.no_grad()
    def _fill_hyper(self, gi, group, advance=True):
        h = self._hyper[gi]
        for j, v in enumerate(self._hyper_values(gi, group, advance)):
            h[j:j + 1].fill_(float(v))

    @torch.no_grad()
    def pre_replay(self):
        for gi, group in enumerate(self.param_groups):
            if gi in self._hyper:
                self._fill_hyper(gi, group)

    # ------------------------------------------------------------------ overlapped step (DDP per bucket)
    # DistributedDataParallel.overlap_optimizer(opt): the update of each gradient bucket is applied on an
    # optimizer stream as soon as the bucket's all-reduce has completed, while the backward of the earlier layers
    # still runs; the step() that follows the backward then has nothing left to do.  One param group on the flat
    # arena, eager (not graph) mode.
    def _overlap_ok(self):
        if self._graph or len(self.param_groups) != 1:
            return None
        fp, rng = self._group_flat(0, self.param_groups[0])
        if fp is None or not fp.data.is_cuda:
            return None
        return fp, rng

    @torch.no_grad()
    def _overlap_begin(self):
        """Host side, once per step before the first range: advance the step state (and create it)."""
        self._ovl_state = self._begin_ranges(0, self.param_groups[0])
        self._ovl_done = False

    @torch.no_grad()
    def _overlap_range(self, a, b):
        """Update flat-arena elements [a, b) (a bucket) with the state _overlap_begin prepared (current stream)."""
        self._apply_range(0, self.param_groups[0], a, b, self._ovl_state)

    def _overlap_end(self):
        fp, _ = self._group_flat(0, self.param_groups[0])
        fp.generation += 1
        self._ovl_done = True          # the next step() finds the update applied

    def _begin_ranges(self, gi, group):
        raise NotImplementedError

    def _apply_range(self, gi, group, a, b, state):
        raise NotImplementedError

    def _consume_overlap(self):
        if getattr(self, "_ovl_done", False):
            self._ovl_done = False
            return True
        return False

    def zero_grad(self, set_to_none: bool = False):
        done = set()
        for group in self.param_groups:
            for p in group["params"]:
                fp = getattr(p, "_pdnn_flat", None)
                if fp is not None:
                    if id(fp) not in done:
                        fp.zero_grad()
                        done.add(id(fp))
                elif p.grad is not None:
                    if set_to_none:
                        p.grad = None
                    else:
                        p.grad.detach_()
                        p.grad.zero_()


class SGD(_FusedBase):
    def __init__(self, params, lr=0.01, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False):
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        super().__init__(params, dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                                      nesterov=nesterov))

    def _check_graphable(self, gi):
        # the first momentum step initialises the buffer (a different kernel branch): run it eagerly
        if self.param_groups[gi]["momentum"] != 0 and "momentum_buffer" not in self.state.get(f"flat{gi}", {}):
            raise RuntimeError("SGD graph mode: run one eager step before capture (momentum buffer init)")

    def _begin_ranges(self, gi, group):
        fp, (s, e) = self._group_flat(gi, group)
        st = self.state.setdefault(f"flat{gi}", {})
        first = "momentum_buffer" not in st
        if group["momentum"] != 0 and first:
            st["momentum_buffer"] = torch.zeros(e - s, device=fp.data.device)
        return first

    def _apply_range(self, gi, group, a, b, first):
        from ..ops import kernels as K
        fp, (s, _) = self._group_flat(gi, group)
        buf = self.state[f"flat{gi}"].get("momentum_buffer")
        K.sgd_step(fp.data[a:b], fp.grad[a:b], None if buf is None else buf[a - s:b - s],
                   fp.shadow[a:b] if fp.shadow is not None else None, group["lr"], group["momentum"],
                   group["dampening"], group["weight_decay"], group["nesterov"], self.grad_scale_dev,
                   self.grad_scale, first)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if self._consume_overlap():
            return loss
        for gi, group in enumerate(self.param_groups):
            lr, mom, damp, wd, nest = (group["lr"], group["momentum"], group["dampening"], group["weight_decay"],
                                       group["nesterov"])
            fp, rng = self._group_flat(gi, group)
            if fp is not None and fp.data.is_cuda:
                from ..ops import kernels as K
                s, e = rng
                st = self.state.setdefault(f"flat{gi}", {})
                first = "momentum_buffer" not in st
                if mom != 0 and first:
                    st["momentum_buffer"] = torch.zeros(e - s, device=fp.data.device)
                buf = st.get("momentum_buffer")
                hyper = self._hyper_buf(gi, 1, fp.data.device) if self._graph else None
                K.sgd_step(fp.data[s:e], fp.grad[s:e], buf, fp.shadow[s:e] if fp.shadow is not None else None,
                           lr, mom, damp, wd, nest, self.grad_scale_dev, self.grad_scale, first, hyper=hyper)
                fp.generation += 1
                continue
            for p in group["params"]:
                if p.grad is None:
                    continue
                g = p.grad
                if self.grad_scale != 1.0:
                    g = g * self.grad_scale
                if self.grad_scale_dev is not None:
                    g = g * self.grad_scale_dev
                if wd != 0:
                    g = g.add(p, alpha=wd)
                if mom != 0:
                    st = self.state[p]
                    if "momentum_buffer" not in st:
                        st["momentum_buffer"] = g.clone().detach()
                    else:
                        st["momentum_buffer"].mul_(mom).add_(g, alpha=1 - damp)
                    b = st["momentum_buffer"]
                    g = g.add(b, alpha=mom) if nest else b
                p.add_(g, alpha=-lr)
        return loss


class Adam(_FusedBase):
    decoupled = False

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))

    _HYPER_LEN = 3

    def _hyper_values(self, gi, group, advance=True):
        st = self.state.setdefault(f"flat{gi}", {})
        if advance:
            st["step"] = st.get("step", 0) + 1       # this replay is step t
        t = max(st.get("step", 0), 1)
        b1, b2 = group["betas"]
        return [group["lr"], 1 - b1 ** t, 1 - b2 ** t]

    def _begin_ranges(self, gi, group):
        fp, (s, e) = self._group_flat(gi, group)
        st = self.state.setdefault(f"flat{gi}", {})
        if "step" not in st:
            st["step"] = 0
            st["exp_avg"] = torch.zeros(e - s, device=fp.data.device)
            st["exp_avg_sq"] = torch.zeros(e - s, device=fp.data.device)
        st["step"] += 1
        return max(st["step"], 1)

    def _apply_range(self, gi, group, a, b, t):
        from ..ops import kernels as K
        fp, (s, _) = self._group_flat(gi, group)
        st = self.state[f"flat{gi}"]
        (b1, b2) = group["betas"]
        K.adam_step(fp.data[a:b], fp.grad[a:b], st["exp_avg"][a - s:b - s], st["exp_avg_sq"][a - s:b - s],
                    fp.shadow[a:b] if fp.shadow is not None else None, group["lr"], b1, b2, group["eps"],
                    group["weight_decay"], self.decoupled, 1 - b1 ** t, 1 - b2 ** t, self.grad_scale_dev,
                    self.grad_scale)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if self._consume_overlap():
            return loss
        for gi, group in enumerate(self.param_groups):
            lr, (b1, b2), eps, wd = group["lr"], group["betas"], group["eps"], group["weight_decay"]
            fp, rng = self._group_flat(gi, group)
            if fp is not None and fp.data.is_cuda:
                from ..ops import kernels as K
                s, e = rng
                st = self.state.setdefault(f"flat{gi}", {})
                if "step" not in st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros(e - s, device=fp.data.device)
                    st["exp_avg_sq"] = torch.zeros(e - s, device=fp.data.device)
                hyper = None
                if self._graph:                  # t advances in pre_replay(); kernel reads hyper[]
                    hyper = self._hyper_buf(gi, 3, fp.data.device)
                else:
                    st["step"] += 1
                t = max(st["step"], 1)
                K.adam_step(fp.data[s:e], fp.grad[s:e], st["exp_avg"], st["exp_avg_sq"],
                            fp.shadow[s:e] if fp.shadow is not None else None, lr, b1, b2, eps, wd,
                            self.decoupled, 1 - b1 ** t, 1 - b2 ** t, self.grad_scale_dev, self.grad_scale,
                            hyper=hyper)
                fp.generation += 1
                continue
            for p in group["params"]:
                if p.grad is None:
                    continue
                g = p.grad * self.grad_scale
                if self.grad_scale_dev is not None:
                    g = g * self.grad_scale_dev
                st = self.state[p]
                if "step" not in st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
                st["step"] += 1
                t = st["step"]
                if self.decoupled:
                    p.mul_(1 - lr * wd)
                elif wd:
                    g = g.add(p, alpha=wd)
                st["exp_avg"].lerp_(g, 1 - b1)
                st["exp_avg_sq"].mul_(b2).addcmul_(g, g, value=1 - b2)
                denom = (st["exp_avg_sq"].sqrt() / math.sqrt(1 - b2 ** t)).add_(eps)    # torch.optim.Adam's order
                p.addcdiv_(st["exp_avg"], denom, value=-lr / (1 - b1 ** t))
        return loss


class AdamW(Adam):
    decoupled = True

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01):
        super().__init__(params, lr, betas, eps, weight_decay)


__all__ = ["SGD", "Adam", "AdamW", "FlatParams"]
