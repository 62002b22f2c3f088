"""Flat parameter arena: every trainable parameter of a model lives in ONE contiguous fp32 buffer.

Why (MI355X-first): with 288 GB of HBM per GPU memory is not the constraint, launch count and
passes over memory are.  A single flat buffer lets

* the optimizer update all parameters in one kernel launch (instead of a per-tensor loop — the
  reference applies updates tensor by tensor: pytorch_code/sync_replicas_master_nn.py:22-28,216-219),
* DDP buckets be zero-copy *views* of the flat gradient buffer (the reference flattens/copies every
  bucket: data_parallel_dist.py:247,262-263),
* the init broadcast be one collective (reference: one broadcast per tensor, data_parallel_dist.py:45-46),
* the bf16 compute shadow of all weights be refreshed in the optimizer pass itself.

Layout: parameters are placed in registration (forward) order, each start aligned to 64 elements
(256 B), 4-D conv weights in channels_last order ([K][R][S][C]) so the shadow slice is exactly what
the implicit-GEMM kernels read.  ``p.data`` / ``p.grad`` become views into ``data`` / ``grad``.
"""
from __future__ import annotations

import os

import torch

from .. import tuning as _tuning

ALIGN = 64
# bumped by every bf16-shadow re-cast issued while a forward may be running (a PS weight bucket landing, an
# on-the-fly re-cast of an externally modified weight): those casts run on the compute stream mid-forward,
# so a side stream that forked from the compute stream earlier in the forward must fork again before it
# reads the shadow (ops/fused_resnet._prep_dgrad_weights)
SHADOW_EPOCH = [0]


def _cl_strides(shape):
    K, C, R, S = shape
    return (R * S * C, 1, S * C, C)


class FlatParams:
    def __init__(self, params, device=None, shadow: bool | None = None, align: int = ALIGN):
        self.params = [p for p in params if p.requires_grad]
        if not self.params:
            raise ValueError("FlatParams: no trainable parameters")
        device = torch.device(device) if device is not None else self.params[0].device
        self.device = device
        self.offsets, off = [], 0
        for p in self.params:
            self.offsets.append(off)
            off += (p.numel() + align - 1) // align * align
        self.numel = off
        self.generation = 0          # bumped by every in-place update of `data` (optimizer step, reload)
        self.data = torch.zeros(off, dtype=torch.float32, device=device)
        self.grad = torch.zeros(off, dtype=torch.float32, device=device)
        use_shadow = (device.type == "cuda") if shadow is None else shadow
        self.shadow = torch.zeros(off, dtype=torch.bfloat16, device=device) if use_shadow else None
        for i, (p, o) in enumerate(zip(self.params, self.offsets)):
            p._pdnn_flat_idx = i
            n = p.numel()
            if p.dim() == 4:
                dv = torch.as_strided(self.data, p.shape, _cl_strides(p.shape), o)
                gv = torch.as_strided(self.grad, p.shape, _cl_strides(p.shape), o)
            else:
                dv = self.data[o:o + n].view(p.shape)
                gv = self.grad[o:o + n].view(p.shape)
            dv.copy_(p.detach().to(device=device, dtype=torch.float32))
            p.data = dv
            p.grad = gv
            p._pdnn_flat = self
            if self.shadow is not None:
                if p.dim() == 4:
                    K, C, R, S = p.shape
                    p._pdnn_shadow = self.shadow[o:o + n].view(K, R, S, C)
                else:
                    p._pdnn_shadow = self.shadow[o:o + n].view(p.shape)
        self.refresh_shadow()

    # ------------------------------------------------------------------
    def refresh_shadow(self):
        """Re-cast the fp32 master weights into the bf16 shadow (after load_state_dict / broadcast)."""
        if self.shadow is None:
            return
        if self.data.is_cuda:
            from ..ops import kernels as K
            K.cast_f32_bf16(self.data, self.shadow)
        else:
            self.shadow.copy_(self.data)
        self.mark_shadow_fresh()

    def refresh_shadow_range(self, start, end):
        """Re-cast one slice [start, end) of the arena (a weight bucket that just arrived) and mark the
        parameters inside it fresh."""
        if self.shadow is None:
            return
        if self.data.is_cuda:
            from ..ops import kernels as K
            K.cast_f32_bf16(self.data[start:end], self.shadow[start:end])
        else:
            self.shadow[start:end].copy_(self.data[start:end])
        self.generation += 1
        SHADOW_EPOCH[0] += 1
        for p, o in zip(self.params, self.offsets):
            if start <= o < end:
                p._pdnn_shadow_ver = p._version

    def mark_shadow_fresh(self):
        self.generation += 1
        for p in self.params:
            p._pdnn_shadow_ver = p._version

    def zero_grad(self):
        self.grad.zero_()
        # a torch optimizer/zero_grad(set_to_none=True) may have detached the views: re-attach
        for p, o in zip(self.params, self.offsets):
            if p.grad is None or p.grad.data_ptr() != self.grad.data_ptr() + 4 * o:
                n = p.numel()
                p.grad = (torch.as_strided(self.grad, p.shape, _cl_strides(p.shape), o) if p.dim() == 4
                          else self.grad[o:o + n].view(p.shape))

    def param_range(self, params):
        """(start, end) of the flat range covering exactly `params` (in arena order), else None."""
        idx = {id(p): i for i, p in enumerate(self.params)}
        ids = [idx.get(id(p)) for p in params]
        if any(i is None for i in ids) or not ids:
            return None
        ids_sorted = sorted(ids)
        if ids_sorted != list(range(ids_sorted[0], ids_sorted[-1] + 1)):
            return None
        start = self.offsets[ids_sorted[0]]
        last = ids_sorted[-1]
        end = self.offsets[last + 1] if last + 1 < len(self.params) else self.numel
        return start, end


def reverse_buckets(fp: FlatParams, cap_mb: float, first_mb: float, early=(), last_mb: float | None = None):
    """Gradient buckets over the flat arena in REVERSE parameter order (the order backward produces
    them), a small first bucket so communication starts early.  -> ([(start, end, n_params)], {id(p): b}).

    ``early``: parameters whose gradient is complete at the START of the backward although they come first in
    arena order (GPT-2's tied token embedding: its LM-head part, once the embedding rows are reduced separately,
    DistributedDataParallel.reduce_sparse_rows).  They form bucket 0, launched as soon as they are ready; they must
    be the leading parameters of the arena (their range and the rest's stay contiguous), else they are ignored.

    ``last_mb``: cap of the LAST bucket (the first layers' gradients, ready only when the backward ends, so its
    collective is the one nothing hides): a larger final group is split so its tail holds at most this much."""
    n = len(fp.params)
    ends = fp.offsets[1:] + [fp.numel]
    pos = {id(q): i for i, q in enumerate(fp.params)}
    lead = sorted(pos[id(q)] for q in early if id(q) in pos)
    if lead != list(range(len(lead))):
        lead = []
    groups, cur, cur_bytes = ([lead] if lead else []), [], 0
    cap = first_mb * 2 ** 20
    for i in reversed(range(len(lead), n)):
        nb = (ends[i] - fp.offsets[i]) * 4
        if cur and cur_bytes + nb > cap:          # close the bucket before it would overflow
            groups.append(cur)
            cur, cur_bytes = [], 0
            cap = cap_mb * 2 ** 20
        cur.append(i)
        cur_bytes += nb
    if cur:
        groups.append(cur)
    if last_mb is not None and len(groups) > (1 if lead else 0):
        last = groups[-1]                     # indices in descending order: the final ones are ready last
        tail, tb = [], 0
        for i in reversed(last):
            nb = (ends[i] - fp.offsets[i]) * 4
            if tail and tb + nb > last_mb * 2 ** 20:
                break
            tail.append(i)
            tb += nb
        if len(tail) < len(last):
            groups[-1] = [i for i in last if i not in set(tail)]
            groups.append(sorted(tail, reverse=True))
    buckets, pbucket = [], {}
    for bi, idxs in enumerate(groups):
        lo, hi = min(idxs), max(idxs)
        buckets.append((fp.offsets[lo], ends[hi], len(idxs)))
        for i in idxs:
            pbucket[id(fp.params[i])] = bi
    return buckets, pbucket


def flatten_module(module: torch.nn.Module, device=None, shadow=None) -> FlatParams:
    """Move ``module``'s trainable parameters into a :class:`FlatParams` arena (idempotent)."""
    fp = getattr(module, "_pdnn_flat", None)
    if fp is not None:
        return fp
    fp = FlatParams(module.parameters(), device=device, shadow=shadow)
    module._pdnn_flat = fp

    def _post_load(mod, incompatible):
        fp.refresh_shadow()
    module.register_load_state_dict_post_hook(_post_load)
    return fp


# ------------------------------------------------------------------------------------------------
# Direct gradient accumulation.  A fused backward op may write a parameter's gradient straight into
# its slice of the flat arena (``p.grad`` is a view of it) instead of returning a fresh tensor that
# autograd's AccumulateGrad then adds in a separate pass: one kernel instead of fill + GEMM + add.
# Such a parameter returns ``None`` from the op's backward.  torch still runs the parameter's
# AccumulateGrad node (a no-op for a None gradient) and its post-accumulate hooks right after the op's
# backward returns, so DDP buckets / PS gradient streaming see it complete at the right time.  Should a
# torch build skip those hooks for None gradients (probed once), :func:`grad_ready` runs them instead.
# Only for parameters used ONCE per forward (a tied weight's contributions are summed by autograd).
# ------------------------------------------------------------------------------------------------
DIRECT_GRAD = True


def await_param(p):
    """Block until ``p``'s weights are current: a PS worker receiving weights bucket by bucket installs
    ``p._pdnn_await`` (parallel/ps.py); everywhere else this is one dict lookup."""
    w = p.__dict__.get("_pdnn_await")
    if w is not None:
        w(p)


class ParamUseMode(torch.overrides.TorchFunctionMode):
    """While active and ``armed()`` is true, every torch op that takes an ``nn.Parameter`` first runs that
    parameter's ``_pdnn_await`` (:func:`await_param`): the per-use hook of torch-op models, whose modules may
    read ``lin.weight`` directly (so module forward hooks never fire).  The fused GPU ops call
    :func:`await_param` themselves when they fetch a weight's bf16 shadow."""

    def __init__(self, armed):
        super().__init__()
        self.armed = armed

    def __torch_function__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if self.armed():
            for a in list(args) + list(kwargs.values()):
                for t in (a if isinstance(a, (list, tuple)) else (a,)):
                    if isinstance(t, torch.nn.Parameter):
                        await_param(t)
        return func(*args, **kwargs)


def direct_grad(p):
    """The arena gradient view of ``p`` if a fused op may accumulate into it directly, else None."""
    if not DIRECT_GRAD or not p.requires_grad:
        return None
    fp = getattr(p, "_pdnn_flat", None)
    g = p.grad
    if fp is None or g is None or not g.is_cuda:
        return None
    if g.data_ptr() != fp.grad.data_ptr() + 4 * fp.offsets[p._pdnn_flat_idx]:
        return None
    return g


_HOOK_ON_NONE = None


def _torch_hooks_fire_on_none() -> bool:
    global _HOOK_ON_NONE
    if _HOOK_ON_NONE is None:
        class _F(torch.autograd.Function):
            @staticmethod
            def forward(ctx, x, w):
                return x * 1

            @staticmethod
            def backward(ctx, g):
                return g, None
        w = torch.nn.Parameter(torch.ones(1))
        x = torch.ones(1, requires_grad=True)
        calls = []
        w.register_post_accumulate_grad_hook(lambda p: calls.append(1))
        _F.apply(x, w).sum().backward()
        _HOOK_ON_NONE = bool(calls)
    return _HOOK_ON_NONE


def grad_ready(p):
    """Announce that a fused op accumulated ``p``'s gradient in place (returns None for it)."""
    if _torch_hooks_fire_on_none():
        return                       # AccumulateGrad will run the hooks after the op's backward
    for fn in getattr(p, "_pdnn_grad_hooks", ()):
        fn(p)


class _GradHookHandle:
    def __init__(self, h, lst, fn):
        self.h, self.lst, self.fn = h, lst, fn

    def remove(self):
        self.h.remove()
        if self.fn in self.lst:
            self.lst.remove(self.fn)


def register_grad_ready_hook(p, fn):
    """``fn(p)`` runs once ``p``'s gradient of the current backward is complete: after AccumulateGrad
    (torch post-accumulate hook) or after a fused op accumulated it in place (:func:`grad_ready`)."""
    h = p.register_post_accumulate_grad_hook(fn)
    lst = p.__dict__.setdefault("_pdnn_grad_hooks", [])
    lst.append(fn)
    return _GradHookHandle(h, lst, fn)


_torch_hooks_fire_on_none()      # probe at import, never from inside a running backward
