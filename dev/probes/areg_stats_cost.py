"""A-stationary 1x1 kernel (conv1x1_panel, conv3x3.hip conv1x1_areg_kernel) on ResNet-50's conv3 forward shapes:
us per call with and without the BN-statistics epilogue (the per-wave fp32 bin atomics), and the data-gradient
form with the residual epilogue."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pytorch_distributed_nn_amd.ops import kernels as K  # noqa: E402

BF = torch.bfloat16


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
    for P, C, N in ((802816, 64, 256), (200704, 128, 512), (50176, 256, 1024), (802816, 256, 64), (50176, 1024, 256)):
        x = torch.randn(P, C, device="cuda").to(BF)
        w = (torch.randn(N, C, device="cuda") * 0.05).to(BF)
        out = {"P": P, "C": C, "N": N, "GB": round((P * C + P * N) * 2 / 1e9, 3)}
        if C > 256:
            print(json.dumps(out), flush=True)
            continue
        out["stats"] = timeit(lambda: K.conv1x1_panel(x, w, want_stats=True))
        out["plain"] = timeit(lambda: K.conv1x1_panel(x, w))
        res = torch.randn(P, N, device="cuda").to(BF)
        out["res"] = timeit(lambda: K.conv1x1_panel(x, w, res=res))
        for k in ("stats", "plain"):
            out[k + "_TBps"] = round(out["GB"] / out[k] * 1e3, 2)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
