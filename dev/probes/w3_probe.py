"""Timing ablations of the direct 3x3 weight-gradient kernel (conv3x3_wgrad.hip; results garbage):
abl 1 = no MFMA, 2 = no halo transpose reads, 4 = no tile loads after the first, combinations."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_nn_amd.ops import kernels as K   # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / iters * 1e3, 1)


for (H, C) in [(56, 64), (28, 128), (14, 256), (7, 512)]:
    N = 256
    x = torch.randn(N, H, H, C, device="cuda").to(torch.bfloat16)
    dy = torch.randn(N, H, H, C, device="cuda").to(torch.bfloat16)
    out = torch.zeros(C, 3, 3, C, device="cuda")
    ws = torch.empty(K.lib().pdnn_conv3x3_wgrad_ws(N, H, H, C, C), device="cuda")
    row = {}
    for abl in [int(v) for v in os.environ.get("W3_ABLS", "0,1,2,3,4,5,6,7").split(",")]:
        K.lib().pdnn_set_w3_ablate(abl)
        row[abl] = timeit(lambda: K.call("pdnn_conv3x3_wgrad", K.ptr(x), K.ptr(dy), K.ptr(out), N, H, H, C, C,
                                         K.ptr(ws), K.stream()))
    K.lib().pdnn_set_w3_ablate(0)
    print(H, C, row, flush=True)
