"""hipBLASLt (torch.matmul) times of the GPT-2 tied LM-head GEMMs, M = 8192 tokens, V = 50304, C = 768."""
import torch


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


M, V, C = 8192, 50304, 768
x = torch.randn(M, C, device="cuda").bfloat16()
w = torch.randn(V, C, device="cuda").bfloat16()
dl = torch.randn(M, V, device="cuda").bfloat16()
f = 2 * M * V * C / 1e6
for name, fn in (("fwd x@w.t()", lambda: x @ w.t()), ("dgrad dl@w", lambda: dl @ w),
                 ("wgrad dl.t()@x (bf16 out)", lambda: dl.t() @ x),
                 ("wgrad fp32 addmm_", lambda: torch.mm(dl.t(), x, out_dtype=torch.float32) if hasattr(torch.mm, "__call__") else None)):
    try:
        us = t(fn)
        print(f"torch {name}: {us:.1f} us {f / us:.0f} TF/s")
    except Exception as ex:  # noqa: BLE001
        print(f"torch {name}: failed {type(ex).__name__}: {ex}")
