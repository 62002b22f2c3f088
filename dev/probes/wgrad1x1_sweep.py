"""ResNet-50 (bs 256) 1x1 weight gradients dW[Cout][Cin] = dy[P][Cout]^T x[P][Cin] on the pp engine: the current
long-reduction split model vs forced tile widths x split counts, us per call including the slab reduction."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pytorch_distributed_nn_amd.ops import kernels as K  # noqa: E402
from pytorch_distributed_nn_amd.ops._backend import lib  # noqa: E402


def t(fn, it=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


SH = (("s2c1", 128, 512, 200704), ("s2c3", 512, 128, 200704), ("s3b1c1", 256, 512, 200704),
      ("s3c1", 256, 1024, 50176), ("s3c3", 1024, 256, 50176), ("s4b1c1", 512, 1024, 50176),
      ("s4c1", 512, 2048, 12544), ("s4c3", 2048, 512, 12544))
for name, M, N, P in SH:
    dy = torch.randn(P, M, device="cuda").bfloat16()
    x = torch.randn(P, N, device="cuda").bfloat16()
    out = torch.zeros(M, N, device="cuda")
    ws = torch.empty(256 * (M * N + 64), device="cuda")
    K.set_pp_bn(0)
    sl = lib().pdnn_pp_wgrad_splits_long(M, N, P)
    plan = lib().pdnn_pp_wgrad_plan(M, N, P, 0)
    row = [f"{name} M={M} N={N} P={P}: long(s={sl})={t(lambda: K.pp_wgrad(dy, x, out, splits=sl, ws=ws)):.1f}",
           f"plan(bn{plan // 1000}s{plan % 1000})={t(lambda: K.pp_wgrad(dy, x, out, ws=ws)):.1f}"]
    nsl = P // 32
    for bn in (128, 256):
        K.set_pp_bn(bn)
        for s in (4, 8, 16, 32, 64, 128, 256):
            if nsl // s < 16:
                continue
            row.append(f"bn{bn}s{s}={t(lambda: K.pp_wgrad(dy, x, out, splits=s, ws=ws)):.1f}")
    K.set_pp_bn(0)
    print(" ".join(row), flush=True)
    del dy, x, out, ws
