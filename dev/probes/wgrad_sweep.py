"""GPT-2 weight-gradient GEMMs (out[M][N] += dY^T X, K = 8192 tokens) on the pp engine: tile width x K-splits sweep,
us per call including the slab reduction, vs the automatic choice and hipBLASLt (fp32 out)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pytorch_distributed_nn_amd.ops import kernels as K  # noqa: E402
from pytorch_distributed_nn_amd.ops._backend import lib  # noqa: E402


def t(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


T = 8192
SW = (1, 2, 3, 4, 6, 8, 12, 16)
for name, M, N, sw in (("qkv", 2304, 768, SW), ("proj", 768, 768, SW), ("fc", 3072, 768, SW), ("fc2", 768, 3072, SW),
                       ("head", 50304, 768, (1, 2, 3))):
    x = torch.randn(T, M, device="cuda").bfloat16()
    y = torch.randn(T, N, device="cuda").bfloat16()
    out = torch.zeros(M, N, device="cuda")
    ws = torch.empty(max(sw) * (M * N + 64), device="cuda")
    K.set_pp_bn(0)
    plan = lib().pdnn_pp_wgrad_plan(M, N, T, 0)
    row = [f"{name} M={M} N={N}: auto(bn{plan // 1000}s{plan % 1000})={t(lambda: K.pp_wgrad(x, y, out, ws=ws)):.1f}"]
    try:
        row.append(f"torch={t(lambda: torch.mm(x.t(), y, out_dtype=torch.float32)):.1f}")
    except Exception:  # noqa: BLE001
        row.append(f"torch_bf16={t(lambda: x.t() @ y):.1f}")
    for bn in (128, 256):
        K.set_pp_bn(bn)
        for s in sw:
            row.append(f"bn{bn}s{s}={t(lambda: K.pp_wgrad(x, y, out, splits=s, ws=ws)):.1f}")
    K.set_pp_bn(0)
    print(" ".join(row), flush=True)
