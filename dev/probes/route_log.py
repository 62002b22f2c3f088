"""Which in-tree kernel entry point every conv / GEMM of a model step calls, with its shape arguments: wraps
ops.kernels.call, runs one warm step of the fused model (bf16, bs from argv), and prints one line per distinct
(entry, integer args) with its count -- the per-layer routing behind a kernel trace's template names.

    python dev/probes/route_log.py [resnet50] [batch]
"""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pytorch_distributed_nn_amd.models import build_model  # noqa: E402
from pytorch_distributed_nn_amd.ops import kernels as K  # noqa: E402
from pytorch_distributed_nn_amd.ops import functional as OF  # noqa: E402
from pytorch_distributed_nn_amd.optim import SGD, flatten_module  # noqa: E402


def main():
    arch = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    model = build_model(arch, num_classes=1000).cuda()
    flatten_module(model)
    opt = SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5)
    x = torch.randn(B, 3, 224, 224, device="cuda").to(torch.bfloat16)
    y = torch.randint(0, 1000, (B,), device="cuda")

    def step():
        opt.zero_grad()
        OF.cross_entropy(model(x), y).backward()
        opt.step()

    step()
    torch.cuda.synchronize()
    log = collections.Counter()
    real = K.call

    def logged(name, *args):
        ints = tuple(a for a in args if isinstance(a, int) and abs(a) < (1 << 31))
        log[(name, ints)] += 1
        return real(name, *args)

    K.call = logged
    try:
        step()
        torch.cuda.synchronize()
    finally:
        K.call = real
    for (name, ints), n in sorted(log.items()):
        print(f"{n:3d}x {name} {ints}")


if __name__ == "__main__":
    main()
