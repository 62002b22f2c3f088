"""StemFn forward outputs: NCHW vs NHWC-direct vs generic (debug)."""
import torch
from pytorch_distributed_nn_amd import tuning
from pytorch_distributed_nn_amd.models import build_model
from pytorch_distributed_nn_amd.ops import kernels as K
from pytorch_distributed_nn_amd.ops import functional as OF
from pytorch_distributed_nn_amd.ops.fused_resnet import StemFn, stem_shadow
from pytorch_distributed_nn_amd.models.resnet import _bn_conf

torch.manual_seed(0)
m = build_model("resnet50").cuda()
g = torch.Generator().manual_seed(5)
x = torch.randn(4, 3, 64, 64, generator=g).cuda().to(torch.bfloat16)
mom, eps = _bn_conf(m.bn1)
conf = (2, 3, True, True, mom, eps)
params = (m.conv1.weight, m.bn1.weight, m.bn1.bias)
outs = {}
for mode in (2, 1, 0):
    tuning.set("stem", mode)
    bufs = [m.bn1.running_mean.clone(), m.bn1.running_var.clone()]
    if mode == 2:
        w = K.stem_weight_nchw(m.conv1.weight)
        y = StemFn.apply(x.contiguous(), conf, bufs, [w], *params)
        print("w32", w.shape, w.float().abs().sum().item())
    else:
        xin = OF.nchw_to_nhwc_input(x)
        ks = stem_shadow(m.conv1.weight, xin.shape[-1])
        print("kpad", ks.shape, ks.float().abs().sum().item(), "wb", m.conv1.weight.to(torch.bfloat16).float().abs().sum().item())
        y = StemFn.apply(xin, conf, bufs, [ks], *params)
    torch.cuda.synchronize()
    outs[mode] = y.float()
    print(mode, y.shape, y.float().abs().mean().item())
for a, b in ((2, 1), (1, 0), (2, 0)):
    d = (outs[a] - outs[b]).abs()
    print(a, b, "max", d.max().item(), "mean", d.mean().item())
