"""Weight gradients of the ResNet-50 1x1 stride-1 convs (bs256): the 128-row implicit-GEMM engine
(K.conv_wgrad, split-K fp32 atomics, im2col B loader) vs the ping-pong engine's plain wgrad (K.pp_wgrad:
dW[Ko][C] = dy[pix][Ko]^T . x[pix][C], split-K slabs + reduce) at several split counts.

    python tools/bench_wgrad1x1.py           -> one JSON line per (stage, conv)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_nn_amd import tuning              # noqa: E402
from pytorch_distributed_nn_amd.ops import kernels as K   # noqa: E402

STAGES = [(56, 64), (28, 128), (14, 256), (7, 512)]


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


def main():
    N = int(os.environ.get("BATCH", "256"))
    d = "cuda"
    for H, C in STAGES:
        for name, cin, ko in (("conv1", 4 * C, C), ("conv3", C, 4 * C)):
            x = torch.randn(N, H, H, cin, device=d).to(torch.bfloat16)
            dy = torch.randn(N, H, H, ko, device=d).to(torch.bfloat16)
            M = N * H * H
            flop = 2.0 * M * cin * ko
            out = torch.zeros(ko, 1, 1, cin, device=d)
            row = {"H": H, "conv": name, "Ko": ko, "C": cin}
            old = tuning.set("wgrad1x1_pp_pix", 0)          # the 128-row implicit-GEMM engine
            row["reg_us"] = timeit(lambda: K.conv_wgrad(x, dy, 1, 1, 1, 0, out=out))
            ref = K.conv_wgrad(x, dy, 1, 1, 1, 0).view(ko, cin)
            tuning.set("wgrad1x1_pp_pix", old)
            o2 = torch.zeros(ko, cin, device=d)
            x2, dy2 = x.view(M, cin), dy.view(M, ko)
            auto = K.lib().pdnn_pp_wgrad_splits_long(ko, cin, M)
            row["pp_auto_splits"] = auto
            best = None
            for s in sorted({auto, 8, 16, 32, 64, 128, 256}):
                ws = torch.empty(s * (ko * cin + 64), device=d)
                t = timeit(lambda: K.pp_wgrad(dy2, x2, o2, splits=s, ws=ws))
                row[f"pp_s{s}_us"] = t
                if best is None or t < best[1]:
                    best = (s, t)
            o2.zero_()
            ws = torch.empty(best[0] * (ko * cin + 64), device=d)
            K.pp_wgrad(dy2, x2, o2, splits=best[0], ws=ws)
            row["pp_best"] = best
            row["rel_err"] = float((o2 - ref).norm() / ref.norm())
            row["reg_TFs"] = round(flop / row["reg_us"] / 1e6, 1)
            row["pp_best_TFs"] = round(flop / best[1] / 1e6, 1)
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
