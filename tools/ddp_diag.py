"""Diagnose DDP-vs-local gradient drift on one GPU: python tools/ddp_diag.py {nccl|gloo|nocomm}
(run under torchrun --nproc-per-node 1 with PDNN_FORCE_PG=1)."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mode = sys.argv[1]
os.environ["PDNN_FORCE_PG"] = "1"
if mode != "nocomm":
    os.environ["PDNN_DDP_FORCE_COMM"] = "1"
from pytorch_distributed_nn_amd.parallel import runtime  # noqa: E402
runtime.init_process_group(backend="gloo" if mode == "gloo" else "nccl")
from pytorch_distributed_nn_amd.models import build_model  # noqa: E402
from pytorch_distributed_nn_amd.ops import functional as OF  # noqa: E402
from pytorch_distributed_nn_amd.optim import SGD  # noqa: E402
from pytorch_distributed_nn_amd.optim.flat import flatten_module  # noqa: E402
from pytorch_distributed_nn_amd.parallel.ddp import DistributedDataParallel  # noqa: E402

torch.manual_seed(0)
dev = torch.device("cuda")
arch = sys.argv[2] if len(sys.argv) > 2 else "resnet50"
m = build_model(arch).to(dev)
ref = copy.deepcopy(m)
fref = flatten_module(ref)
net = DistributedDataParallel(m, bucket_cap_mb=4.0, first_bucket_cap_mb=0.5)
print("comm", net._comm, "nccl", net.nccl, "buckets", len(net.buckets))
lr = float(os.environ.get("DIAG_LR", "0.05"))
opt, opt_ref = SGD(m.parameters(), lr=lr, momentum=0.9), SGD(ref.parameters(), lr=lr, momentum=0.9)
g = torch.Generator().manual_seed(1)
prev = None
for it in range(3):
    x, y = torch.randn(4, 3, 64, 64, generator=g).to(dev), torch.randint(0, 1000, (4,), generator=g).to(dev)
    for n, o in ((net, opt), (ref, opt_ref)):
        o.zero_grad()
        OF.cross_entropy(n(x), y).backward()
        torch.cuda.synchronize()
        if n is net:
            gn = net.flat.grad.clone()
        o.step()
    torch.cuda.synchronize()
    gr = fref.grad
    rel = ((gn - gr).norm() / gr.norm()).item()
    relp = ((net.flat.data - fref.data).norm() / fref.data.norm()).item()
    msg = f"step {it}: grad rel {rel:.3e} param rel {relp:.3e} |gn| {gn.norm():.4f} |gr| {gr.norm():.4f}"
    if prev is not None:
        msg += f" rel(gn, gr+prev) {((gn - gr - prev).norm() / gr.norm()).item():.3e}"
    # which parameters differ most
    worst = []
    for i, p in enumerate(fref.params):
        s = fref.offsets[i]
        e = s + p.numel()
        d = ((gn[s:e] - gr[s:e]).norm() / (gr[s:e].norm() + 1e-12)).item()
        worst.append((d, i, tuple(p.shape)))
    worst.sort(reverse=True)
    print(msg, "worst", worst[:4], flush=True)
    prev = gr.clone()
runtime.destroy()
