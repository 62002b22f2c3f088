"""Per-parameter gradient comparison of ResNet-50 with tuning stem = 1 vs 0 (debug)."""
import torch
from pytorch_distributed_nn_amd import tuning
from pytorch_distributed_nn_amd.models import build_model
from pytorch_distributed_nn_amd.ops import functional as OF
from pytorch_distributed_nn_amd.optim import flatten_module


def grads(flat):
    torch.manual_seed(0)
    m = build_model("resnet50").cuda()
    fp = flatten_module(m) if flat else None
    g = torch.Generator().manual_seed(5)
    x = torch.randn(4, 3, 64, 64, generator=g).cuda().to(torch.bfloat16)
    y = torch.randint(0, 1000, (4,), generator=g).cuda()
    if fp is not None:
        fp.zero_grad()
    else:
        m.zero_grad(set_to_none=True)
    loss = OF.cross_entropy(m(x), y)
    loss.backward()
    torch.cuda.synchronize()
    return loss.item(), {n: p.grad.detach().float().clone() for n, p in m.named_parameters() if p.grad is not None}


for modes in ((2, 1), (1, 0), (2, 0)):
    res = []
    for mode in modes:
        tuning.set("stem", mode)
        res.append(grads(False))
    cs = []
    for n in res[0][1]:
        a, b = res[0][1][n], res[1][1][n]
        cs.append((torch.nn.functional.cosine_similarity(a.flatten(), b.flatten(), dim=0).item(), n))
    cs.sort()
    print(modes, "loss", res[0][0], res[1][0], "worst", cs[:3], "conv1", [c for c in cs if c[1] == "conv1.weight"])
