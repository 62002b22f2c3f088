"""GPT-2 LayerNorm kernels at 8192 x 768 (bf16): forward, and backward (with the residual-gradient add) per block
count; us per call and effective HBM bandwidth."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pytorch_distributed_nn_amd.ops import kernels as K  # noqa: E402
from pytorch_distributed_nn_amd.ops._backend import lib  # noqa: E402


def t(fn, it=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


R, D = 8192, 768
x = torch.randn(R, D, device="cuda").bfloat16()
dy = torch.randn(R, D, device="cuda").bfloat16()
dres = torch.randn(R, D, device="cuda").bfloat16()
g = torch.rand(D, device="cuda") + 0.5
b = torch.randn(D, device="cuda")
y, mean, rstd = K.layernorm_fwd(x, g, b, 1e-5)
us = t(lambda: K.layernorm_fwd(x, g, b, 1e-5))
print(f"fwd {us:.1f} us {R * D * 4 / us / 1e3:.2f} TB/s")
slab = K.stat_bins(D, x.device)
dx = torch.empty_like(x)
for nb in (64, 128, 256, 512):
    fn = lambda: K.call("pdnn_layernorm_bwd", K.ptr(dy), K.ptr(x), K.ptr(g), K.ptr(mean), K.ptr(rstd),  # noqa: E731
                        K.ptr(dres), K.ptr(dx), K.ptr(slab), R, D, nb, K.stream())
    us = t(fn)
    print(f"bwd nblocks={nb} {us:.1f} us {R * D * 8 / us / 1e3:.2f} TB/s", flush=True)
print("auto nblocks", lib().pdnn_layernorm_bwd_blocks(R))
