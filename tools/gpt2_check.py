"""Diagnostic: fused GPU GPT-2 vs the fp32 PyTorch reference path on the same GPU (grads + loss curves)."""
import copy
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_nn_amd.models.gpt2 import build_gpt2  # noqa: E402
from pytorch_distributed_nn_amd.optim import AdamW, flatten_module  # noqa: E402


def main():
    L = int(os.environ.get("LAYERS", "12"))
    B, T = int(os.environ.get("B", "4")), 1024
    torch.manual_seed(0)
    m = build_gpt2("gpt2_small", n_layer=L).cuda()
    ref = copy.deepcopy(m)
    toks = torch.randint(0, 50257, (B, T + 1), device="cuda")
    x, y = toks[:, :-1].contiguous(), toks[:, 1:].contiguous()
    loss = m(x, y)
    loss.backward()
    lr = ref._forward_reference(x, y)
    lr.backward()
    print(f"loss fused {loss.item():.5f} ref {lr.item():.5f}")
    for (n, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
        c = F.cosine_similarity(p.grad.flatten().float(), q.grad.flatten().float(), dim=0).item()
        r = ((p.grad - q.grad).norm() / q.grad.norm().clamp_min(1e-20)).item()
        flag = "  <-- BAD" if c < 0.98 else ""
        print(f"{n:45s} cos {c:.5f} rel {r:.4f} |g| {p.grad.norm().item():.3e} ref {q.grad.norm().item():.3e}{flag}")
    # training curves
    m.zero_grad(set_to_none=True)
    ref.zero_grad(set_to_none=True)
    flatten_module(m)
    o1 = AdamW(m.parameters(), lr=6e-4, betas=(0.9, 0.95), weight_decay=0.1)
    o2 = torch.optim.AdamW(ref.parameters(), lr=6e-4, betas=(0.9, 0.95), weight_decay=0.1)
    for i in range(15):
        o1.zero_grad()
        a = m(x, y)
        a.backward()
        o1.step()
        o2.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            b = ref._forward_reference(x, y)
        b.backward()
        o2.step()
        print(f"step {i} fused {a.item():.4f} ref(autocast) {b.item():.4f}")


if __name__ == "__main__":
    main()
