"""Per-layer timing of the 1x1 convs of the ResNet-50 bottleneck (bs256) as the fused block runs them:
conv3 forward with the BN2+ReLU operand prologue vs materialised a2 = relu(bn2(t2)) (bn_apply) + plain
conv, conv1 forward with BN statistics, conv3 data gradient with the BN-backward epilogue and conv1 data
gradient with the residual.  Engine choice comes from the dispatch table (PDNN_TUNE="pp_conv_fwd_k=0,pp_conv_bnb_k=0",
csrc/kernels/tuning.h), so one call per configuration.

    PDNN_TUNE=pp_conv_fwd_k=0 python tools/bench_conv1x1.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_nn_amd.ops import kernels as K   # noqa: E402

# (H, C_mid, count): input/output channels 4*C_mid
STAGES = [(56, 64, 3), (28, 128, 4), (14, 256, 6), (7, 512, 3)]


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
    tot = {}
    tag = {k: v for k, v in os.environ.items() if k.startswith("PDNN_")}
    for H, C, cnt in STAGES:
        C4 = 4 * C
        d = "cuda"
        t2 = torch.randn(N, H, H, C, device=d).to(torch.bfloat16)
        x4 = torch.randn(N, H, H, C4, device=d).to(torch.bfloat16)
        k3 = (torch.randn(C4, 1, 1, C, device=d) * 0.05).to(torch.bfloat16)
        k1 = (torch.randn(C, 1, 1, C4, device=d) * 0.05).to(torch.bfloat16)
        sc, sh = torch.rand(C, device=d) + 0.5, torch.randn(C, device=d) * 0.1
        mean, inv = torch.zeros(C, device=d), torch.ones(C, device=d)
        dt3 = torch.randn(N, H, H, C4, device=d).to(torch.bfloat16)
        dt1 = torch.randn(N, H, H, C, device=d).to(torch.bfloat16)
        row = {"H": H, "C": C}
        row["conv3_fwd_pro"] = timeit(lambda: K.conv_fwd(t2, k3, 1, 0, pro=(sc, sh), want_stats=True))
        row["bn_apply_a2"] = timeit(lambda: K.bn_apply(t2.view(-1, C), sc, sh, relu=True))
        a2 = K.bn_apply(t2.view(-1, C), sc, sh, relu=True).view(t2.shape)
        row["conv3_fwd_plain"] = timeit(lambda: K.conv_fwd(a2, k3, 1, 0, want_stats=True))
        row["conv1_fwd"] = timeit(lambda: K.conv_fwd(x4, k1, 1, 0, want_stats=True))
        row["conv3_dgrad_bn"] = timeit(lambda: K.conv_dgrad(dt3, k3, t2.shape, 1, 0, bn=(t2, mean, inv, sc, sh)))
        # the BN3 backward apply pass that produces dt3 from the block output's gradient
        t3 = torch.randn(N, H, H, C4, device=d).to(torch.bfloat16)
        ob = torch.randint(0, 256, (N * H * H, C4 // 8), device=d, dtype=torch.uint8)
        m3, i3, g3 = torch.zeros(C4, device=d), torch.ones(C4, device=d), torch.rand(C4, device=d) + 0.5
        dg3, db3 = torch.randn(C4, device=d), torch.randn(C4, device=d)
        row["bn3_apply"] = timeit(lambda: K.bn_bwd_apply(dt3.view(-1, C4), t3.view(-1, C4), m3, i3, g3, dg3, db3,
                                                         mode=3, msrc=ob))
        row["conv1_dgrad_res"] = timeit(lambda: K.conv_dgrad(dt1, k1, x4.shape, 1, 0, res=x4))
        bits = torch.randint(0, 256, (N * H * H, C4 // 8), device=d, dtype=torch.uint8)
        row["conv1_dgrad_res_mask"] = timeit(lambda: K.conv_dgrad(dt1, k1, x4.shape, 1, 0, res=x4, res_mask=bits))
        if K.dgrad_pre_ok(dt1.shape, k1.shape, 1, 0):
            # the Bottleneck's conv1 data gradient: BN1's backward apply in the operand loads, dt1 written
            g1, dg, db = torch.rand(C, device=d) + 0.5, torch.randn(C, device=d), torch.randn(C, device=d)
            dt_out = torch.empty_like(dt1)
            pre = (t2, mean, inv, g1, dg, db, dt_out)
            row["conv1_dgrad_pre"] = timeit(lambda: K.conv_dgrad(dt1, k1, x4.shape, 1, 0, pre=pre))
            row["conv1_dgrad_pre_res_mask"] = timeit(
                lambda: K.conv_dgrad(dt1, k1, x4.shape, 1, 0, res=x4, res_mask=bits, pre=pre))
            row["conv1_dgrad_pre_nowrite"] = timeit(
                lambda: K.conv_dgrad(dt1, k1, x4.shape, 1, 0, res=x4, res_mask=bits, pre=pre[:6] + (None,)))
        print(json.dumps(row), flush=True)
        for k, v in row.items():
            if k not in ("H", "C"):
                tot[k] = round(tot.get(k, 0.0) + cnt * v, 1)
    print(json.dumps({"env": tag, "per_step_us": tot}), flush=True)


if __name__ == "__main__":
    main()
