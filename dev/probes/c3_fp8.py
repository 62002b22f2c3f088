"""fp8 vs bf16 halo 3x3 conv at the ResNet-50/152 stage shapes (bs 256): forward with BN statistics and the data
gradient with the BN-backward operand prologue + fused BN-backward epilogue.  us per call (fp8 includes its
scale-roll launch)."""
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
    BF = torch.bfloat16
    for (N, H, C) in [(256, 28, 128), (256, 14, 256)]:
        x = torch.randn(N, H, H, C, device="cuda").to(BF)
        w = (torch.randn(C, 3, 3, C, device="cuda") * 0.05).to(BF)
        winv = torch.empty(1, device="cuda")
        wq = K.quant_fp8_current(w.reshape(C, -1).contiguous(), winv)
        wt = K.conv3x3_flip8(wq, C, C)
        wtb = K.conv3x3_flip(w)
        act, actb = Fp8Act(x.device), Fp8Act(x.device, e5m2=True)
        t = torch.randn_like(x)
        mean, inv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        g, dg, db = torch.ones(C, device="cuda"), torch.randn(C, device="cuda"), torch.randn(C, device="cuda")
        sc, sh = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
        dt = torch.empty_like(x)
        pre = (t, mean, inv, g, dg, db, dt)
        bn = (t, mean, inv, sc, sh)
        out = {"shape": [N, H, H, C, C], "gflop": round(2 * N * H * H * C * C * 9 / 1e9, 1)}
        out["fwd_bf16"] = timeit(lambda: K.conv3x3(x, w, want_stats=True))
        out["fwd_fp8"] = timeit(lambda: K.conv3x3_fp8(x, wq, winv, act, want_stats=True))
        out["dgrad_bf16"] = timeit(lambda: K.conv3x3(x, wtb, bn=bn, pre=pre))
        out["dgrad_fp8"] = timeit(lambda: K.conv3x3_fp8(x, wt, winv, actb, bn=bn, pre=pre))
        out["weight_quant"] = timeit(lambda: K.quant_fp8_current(w.reshape(C, -1).contiguous(), winv))
        out["flip8"] = timeit(lambda: K.conv3x3_flip8(wq, C, C))
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
