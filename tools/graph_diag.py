"""Variants of a captured LeNet training step (diagnosing a host crash at hipGraph capture_end).

    python tools/graph_diag.py --batch 64 --style forward|loss_fn --warmup 2
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--style", default="forward")
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--model", default="LeNet")
    a = ap.parse_args()
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.ops import functional as OF
    from pytorch_distributed_nn_amd.optim import SGD, flatten_module
    from pytorch_distributed_nn_amd.utils.graphs import GraphedStep
    torch.manual_seed(0)
    m = build_model(a.model, 10).cuda()
    flatten_module(m)
    o = SGD(m.parameters(), lr=0.05, momentum=0.9)
    shp = (1, 28, 28) if a.model == "LeNet" else (3, 32, 32)
    x, y = torch.randn(a.batch, *shp).cuda(), torch.randint(0, 10, (a.batch,)).cuda()
    if a.style == "forward":
        gs = GraphedStep(m, o, forward=lambda mm, xx, yy: OF.cross_entropy(mm(xx), yy), warmup=a.warmup)
    else:
        gs = GraphedStep(m, o, loss_fn=OF.cross_entropy, warmup=a.warmup)
    for i in range(a.warmup + 3):
        print(i, float(gs(x, y)), flush=True)
    print("OK", vars(a), flush=True)


if __name__ == "__main__":
    main()
