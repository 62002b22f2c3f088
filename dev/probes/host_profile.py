"""cProfile of the host side of the ResNet-50 bs256 DDP-path step (bench.py's setup at world 1): where the
Python issue time goes, sorted by own time."""
import cProfile
import os
import pstats
import sys

import torch

sys.path.insert(0, os.getcwd())
os.environ.setdefault("PDNN_FORCE_PG", "1")
os.environ.setdefault("PDNN_DDP_FORCE_COMM", "1")
from pytorch_distributed_nn_amd.parallel import runtime  # noqa: E402
from pytorch_distributed_nn_amd.parallel.ddp import DistributedDataParallel  # noqa: E402
from pytorch_distributed_nn_amd.models import build_model  # noqa: E402
from pytorch_distributed_nn_amd.optim import SGD  # noqa: E402
from pytorch_distributed_nn_amd.ops import functional as OF  # noqa: E402

runtime.init_process_group()
dev = runtime.device()
model = build_model("resnet50").to(dev)
net = DistributedDataParallel(model, bucket_cap_mb=32)
opt = SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5)
x = torch.randn(256, 3, 224, 224, device=dev).to(torch.bfloat16)
y = torch.randint(0, 1000, (256,), device=dev)
ms = torch.cuda.Stream(device=dev, priority=-1)
ms.wait_stream(torch.cuda.current_stream(dev))


def step():
    opt.zero_grad()
    OF.cross_entropy(net(x), y).backward()
    opt.step()


with torch.cuda.stream(ms):
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(10):
        step()
    pr.disable()
    torch.cuda.synchronize()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(45)
runtime.destroy()
