"""Host-side launch cost of one training step vs its GPU time (is the step launch-bound?).

With 8 ranks on one node every rank's Python thread must enqueue ~1400 kernels per ResNet-50 step; if that
host time approaches the GPU time, the GPU idles between kernels and multi-GPU scaling suffers.  This
measures, for the bench.py step of ``--model``:

* ``host_ms``: wall time for ``step()`` to *return* right after a device sync (pure enqueue cost, the GPU
  starts idle so nothing back-pressures the launch queue),
* ``gpu_ms``: steady-state time per step (sync-bracketed loop),
* ``launches``: kernels per step (from torch.profiler, when available).

    python tools/host_overhead.py --model resnet50
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.optim import SGD, AdamW, flatten_module
    from pytorch_distributed_nn_amd.ops import functional as OF
    dev = torch.device("cuda")
    lm = a.model.startswith("gpt2")
    m = build_model(a.model, num_classes=1000).to(dev)
    flatten_module(m)
    if lm:
        B = a.batch or 8
        opt = AdamW(m.parameters(), lr=6e-4)
        t = torch.randint(0, 50257, (B, 1025), device=dev)
        x, y = t[:, :-1].contiguous(), t[:, 1:].contiguous()
    else:
        B = a.batch or 256
        opt = SGD(m.parameters(), lr=0.1, momentum=0.9)
        x = torch.randn(B, 3, 224, 224, device=dev).to(torch.bfloat16)
        y = torch.randint(0, 1000, (B,), device=dev)

    def step():
        opt.zero_grad()
        loss = m(x, y) if lm else OF.cross_entropy(m(x), y)
        loss.backward()
        opt.step()

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    host = []
    for _ in range(a.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step()
        host.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    gpu = (time.perf_counter() - t0) / a.steps
    launches = None
    try:
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CUDA]) as p:
            step()
            torch.cuda.synchronize()
        launches = sum(1 for e in p.events() if e.device_type == torch.autograd.DeviceType.CUDA)
    except Exception:
        pass
    host.sort()
    print(json.dumps({"model": a.model, "batch": B, "host_ms_median": round(1e3 * host[len(host) // 2], 3),
                      "host_ms_min": round(1e3 * host[0], 3), "gpu_ms": round(1e3 * gpu, 3),
                      "host_over_gpu": round(host[len(host) // 2] / gpu, 3), "gpu_kernels_per_step": launches}))


if __name__ == "__main__":
    main()
