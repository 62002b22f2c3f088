"""GPT-2 small, 8 AdamW steps on two fixed batches (bench.py's setup; plain step, then the DDP path over a 1-rank
RCCL group with --ddp): per-step losses with the one-pass cross-entropy on / off, twice each."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pytorch_distributed_nn_amd import tuning  # noqa: E402
from pytorch_distributed_nn_amd.models import build_model  # noqa: E402
from pytorch_distributed_nn_amd.optim import AdamW, flatten_module  # noqa: E402


DDP = "--ddp" in sys.argv
if DDP:
    os.environ.setdefault("PDNN_FORCE_PG", "1")
    os.environ.setdefault("PDNN_DDP_FORCE_COMM", "1")
    from pytorch_distributed_nn_amd.parallel import runtime
    from pytorch_distributed_nn_amd.parallel.ddp import DistributedDataParallel
    runtime.init_process_group()


def run(fused):
    tuning.set("xent_fused", fused)
    torch.manual_seed(1234)
    model = build_model("gpt2").cuda()
    if DDP:
        m = DistributedDataParallel(model, bucket_cap_mb=32.0)
    else:
        flatten_module(model)
        m = model
    opt = AdamW(model.parameters(), lr=6e-4, betas=(0.9, 0.95), weight_decay=0.1)
    toks = [torch.randint(0, 50257, (8, 1025), device="cuda") for _ in range(2)]
    out = []
    for i in range(28):             # bench.py's 8 + 20 steps, the host running ahead (no per-step sync)
        t = toks[i % 2]
        opt.zero_grad()
        loss = m(t[:, :-1].contiguous(), t[:, 1:].contiguous())
        loss.backward()
        opt.step()
        out.append(loss.detach())
    return [round(v.item(), 4) for v in out[::3]]


for f in (1, 1, 0, 0):
    print("fused" if f else "two-pass", run(f), flush=True)
