"""fp8 vs bf16 direct 3x3 weight gradient at the ResNet stage shapes (bs 256), us per call."""
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
    from pytorch_distributed_nn_amd.ops.fp8 import Fp8Act
    for (H, C) in [(56, 64), (28, 128), (14, 256), (7, 512)]:
        x = torch.randn(256, H, H, C, device="cuda").to(torch.bfloat16)
        dy = torch.randn(256, H, H, C, device="cuda").to(torch.bfloat16)
        out = torch.zeros(C, 3, 3, C, device="cuda")
        ax, ad = Fp8Act(x.device), Fp8Act(x.device, e5m2=True)
        ax.scale.fill_(100.0); ad.scale.fill_(100.0)
        r = {"shape": [256, H, H, C, C], "bf16": timeit(lambda: K.conv_wgrad(x, dy, 3, 3, 1, 1, out=out)),
             "fp8": timeit(lambda: K.conv3x3_wgrad_fp8(x, dy, ax, ad, out=out))}
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
