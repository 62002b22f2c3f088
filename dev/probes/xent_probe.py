"""GPT-2 head cross-entropy forward: with the per-row same-address loss / count atomics vs without (loss_sum = null),
and the backward pass, us per call at [8192, 50304] bf16."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / iters * 1e3, 1)


def main():
    from pytorch_distributed_nn_amd.ops import kernels as K
    R, V = 8192, 50304
    x = torch.randn(R, V, device="cuda").to(torch.bfloat16)
    y = torch.randint(0, 50257, (R,), device="cuda")
    loss = torch.empty(R, device="cuda")
    lse = torch.empty(R, device="cuda")
    acc = torch.zeros(2, device="cuda")
    g = torch.ones(1, device="cuda")
    out = {"fwd": timeit(lambda: K.xent_fwd(x, y)),
           "fwd_no_atomics": timeit(lambda: K.call("pdnn_xent_fwd", K.ptr(x), x.stride(0), R, V, K.ptr(y), -100,
                                                   K.ptr(loss), K.ptr(lse), None, None, 1, K.stream())),
           "bwd": timeit(lambda: K.xent_bwd(x, y, lse, g, float(R))),
           "torch_logsumexp": timeit(lambda: torch.logsumexp(x.float(), 1) if False else x.amax(1))}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
