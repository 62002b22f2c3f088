"""Stock PyTorch-ROCm comparison line for GPT-2 small (BASELINE.json config 4).

Plain ``torch.nn`` GPT-2 (12L/12H/768, T=1024, vocab 50304, tied head), autocast bf16,
``F.scaled_dot_product_attention`` (ROCm flash/efficient attention backends), fused ``torch.optim.AdamW``.
Prints one JSON line with tokens/sec — the number ``bench.py --model gpt2_small`` has to beat.

    python tools/stock_gpt2.py --batch 8 --steps 10 --warmup 3
"""
import argparse
import json
import math
import time

import torch
import torch.nn as nn
import torch.nn.functional as F


class Block(nn.Module):
    def __init__(self, d, h):
        super().__init__()
        self.h = h
        self.ln_1, self.ln_2 = nn.LayerNorm(d), nn.LayerNorm(d)
        self.c_attn, self.c_proj = nn.Linear(d, 3 * d), nn.Linear(d, d)
        self.c_fc, self.c_fc2 = nn.Linear(d, 4 * d), nn.Linear(4 * d, d)

    def forward(self, x):
        B, T, D = x.shape
        q, k, v = self.c_attn(self.ln_1(x)).split(D, 2)
        q, k, v = (t.view(B, T, self.h, D // self.h).transpose(1, 2) for t in (q, k, v))
        y = F.scaled_dot_product_attention(q, k, v, is_causal=True).transpose(1, 2).reshape(B, T, D)
        x = x + self.c_proj(y)
        return x + self.c_fc2(F.gelu(self.c_fc(self.ln_2(x)), approximate="tanh"))


class GPT(nn.Module):
    def __init__(self, V=50304, T=1024, L=12, H=12, D=768):
        super().__init__()
        self.wte, self.wpe = nn.Embedding(V, D), nn.Embedding(T, D)
        self.h = nn.ModuleList(Block(D, H) for _ in range(L))
        self.ln_f = nn.LayerNorm(D)
        self.head = nn.Linear(D, V, bias=False)
        self.head.weight = self.wte.weight
        for m in self.modules():
            if isinstance(m, (nn.Linear, nn.Embedding)):
                nn.init.normal_(m.weight, 0, 0.02)

    def forward(self, idx, tgt):
        T = idx.shape[1]
        x = self.wte(idx) + self.wpe(torch.arange(T, device=idx.device))
        for b in self.h:
            x = b(x)
        logits = self.head(self.ln_f(x))
        return F.cross_entropy(logits.float().view(-1, logits.shape[-1]), tgt.view(-1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--seq-len", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda")
    m = GPT().to(dev)
    opt = torch.optim.AdamW(m.parameters(), lr=6e-4, betas=(0.9, 0.95), weight_decay=0.1, fused=True)
    t = torch.randint(0, 50257, (a.batch, a.seq_len + 1), device=dev)
    x, y = t[:, :-1].contiguous(), t[:, 1:].contiguous()

    def step():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = m(x, y)
        loss.backward()
        opt.step()
        return loss

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    tok = a.batch * a.seq_len * a.steps / dt
    print(json.dumps({"metric": "tokens/sec stock PyTorch-ROCm GPT-2 small (autocast bf16, SDPA, fused AdamW)",
                      "value": round(tok, 1), "ms_per_step": round(1e3 * dt / a.steps, 3), "batch": a.batch,
                      "seq_len": a.seq_len, "final_loss": round(loss.item(), 4)}), flush=True)


if __name__ == "__main__":
    main()
