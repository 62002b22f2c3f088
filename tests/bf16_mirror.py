"""An fp32 CPU reference that rounds to bf16 at the same points as the fused GPU kernels.

The HIP path keeps fp32 master weights but computes with their bf16 shadow, reads bf16 activations,
accumulates in fp32 and stores every conv / GEMM output, BN+ReLU output and data gradient in bf16.
Comparing it to a plain fp32 reference mixes kernel errors with the (legitimate) bf16 storage noise,
which is large in deep nets at small batch.  This mirror rounds the reference at those points —
weights and input once, every Conv2d / Linear / BatchNorm2d / ReLU / pooling output in the forward and the
gradient flowing into each of them in the backward — so the remaining difference measures the kernels
(accumulation order, fused-epilogue arithmetic, ReLU-mask ties), not the storage format."""
import copy

import torch

BF = torch.bfloat16


class _Round(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return x.to(BF).float()

    @staticmethod
    def backward(ctx, g):
        return g.to(BF).float()


def round_bf16(x):
    return _Round.apply(x)


_ROUNDED = (torch.nn.Conv2d, torch.nn.Linear, torch.nn.BatchNorm2d, torch.nn.ReLU, torch.nn.MaxPool2d,
            torch.nn.AvgPool2d, torch.nn.AdaptiveAvgPool2d)


def mirror(model):
    """fp32 copy of ``model`` with bf16-rounded weights and bf16 rounding at every kernel boundary."""
    ref = copy.deepcopy(model).float().cpu()
    with torch.no_grad():
        for p in ref.parameters():
            if p.dim() > 1:                       # GEMM / conv weights are read from the bf16 shadow
                p.copy_(p.to(BF).float())
    for m in ref.modules():
        if isinstance(m, _ROUNDED):
            m.register_forward_hook(lambda mod, inp, out: round_bf16(out))
    return ref


def rel(a, b):
    a, b = a.float().cpu().flatten(), b.float().cpu().flatten()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def cos(a, b):
    return torch.nn.functional.cosine_similarity(a.float().cpu().flatten(), b.float().cpu().flatten(), dim=0).item()
