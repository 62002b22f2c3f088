"""Stem conv: NCHW kernel vs NHWC kernel vs generic engine vs fp32 (debug)."""
import torch
import torch.nn.functional as F
from pytorch_distributed_nn_amd.ops import kernels as K

torch.manual_seed(0)
for (N, H, W) in [(4, 64, 64), (2, 224, 224)]:
    x = torch.randn(N, 3, H, W, device="cuda").to(torch.bfloat16)
    w = torch.randn(64, 3, 7, 7, device="cuda") * 0.1
    wb = w.to(torch.bfloat16)
    ref = F.conv2d(x.float(), wb.float(), None, 2, 3).permute(0, 2, 3, 1)
    yn, _ = K.stem_conv_nchw(x, K.stem_weight_nchw(w))
    xin = K.nchw_to_nhwc(x, 8)
    kpad = torch.nn.functional.pad(wb.permute(0, 2, 3, 1), (0, 5)).contiguous()
    yh, _ = K.stem_conv(xin, kpad)
    yg, _ = K.conv_fwd(xin, kpad, 2, 3, want_stats=True)
    for name, y in (("nchw", yn), ("nhwc", yh), ("generic", yg)):
        d = (y.float() - ref)
        print(N, H, W, name, "max", d.abs().max().item(), "mean", d.abs().mean().item(), "refmax", ref.abs().max().item(),
              "argmax", torch.nonzero(d.abs() == d.abs().max())[0].tolist())
