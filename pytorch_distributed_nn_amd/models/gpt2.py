"""GPT-2 (BASELINE.json config 4: "GPT-2-small transformer DDP bf16").  New capability — the reference
trains only CNNs/MLPs — built on the same engine: flat fp32 parameter arena with bf16
shadows (``optim.flat``), RCCL DDP buckets (``parallel.ddp``), fused optimizers.

Architecture = GPT-2 small: 12 layers, 12 heads, d_model 768, context 1024, pre-LN blocks, GELU(tanh)
MLP 4x, learned position embeddings, LM head tied to the token embedding.  The vocabulary is padded from
50257 to 50304 (a multiple of 128: MFMA tile-aligned; the extra rows are never targets).  Parameter names
follow the HuggingFace layout (``transformer.h.0.attn.c_attn.weight`` ...), but Linear weights are stored
[out][in] (nn.Linear), i.e. transposed relative to HF's Conv1D.

GPU path: ``ops.transformer`` fused Functions (one autograd node per block); CPU path: plain PyTorch in
fp32 (tests, and the numerics reference of the GPU path).  ``forward(idx, targets)`` returns the mean
next-token cross-entropy when targets are given (the fused head never materialises fp32 logits),
otherwise the logits.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import tuning
from ..ops import functional as OF
from ..ops import transformer as TX
from ..optim.flat import direct_grad


@dataclass
class GPT2Config:
    vocab_size: int = 50304
    block_size: int = 1024
    n_layer: int = 12
    n_head: int = 12
    n_embd: int = 768
    eps: float = 1e-5
    fp8: bool = False          # block linears' forward GEMMs in fp8 (e4m3, delayed scaling); bwd bf16


CONFIGS = {
    "gpt2_small": GPT2Config(),
    "gpt2": GPT2Config(),
    "gpt2_medium": GPT2Config(n_layer=24, n_head=16, n_embd=1024),
    "gpt2_large": GPT2Config(n_layer=36, n_head=20, n_embd=1280),
    "gpt2_tiny": GPT2Config(vocab_size=512, block_size=128, n_layer=2, n_head=2, n_embd=128),
}


class Attention(nn.Module):
    def __init__(self, c: GPT2Config):
        super().__init__()
        self.n_head = c.n_head
        self.c_attn = nn.Linear(c.n_embd, 3 * c.n_embd)
        self.c_proj = nn.Linear(c.n_embd, c.n_embd)

    def forward(self, x):
        B, T, D = x.shape
        q, k, v = self.c_attn(x).split(D, dim=2)
        q, k, v = (t.view(B, T, self.n_head, D // self.n_head).transpose(1, 2) for t in (q, k, v))
        y = F.scaled_dot_product_attention(q, k, v, is_causal=True)
        return self.c_proj(y.transpose(1, 2).reshape(B, T, D))


class MLP(nn.Module):
    def __init__(self, c: GPT2Config):
        super().__init__()
        self.c_fc = nn.Linear(c.n_embd, 4 * c.n_embd)
        self.c_proj = nn.Linear(4 * c.n_embd, c.n_embd)

    def forward(self, x):
        return self.c_proj(F.gelu(self.c_fc(x), approximate="tanh"))


class Block(nn.Module):
    def __init__(self, c: GPT2Config):
        super().__init__()
        self.ln_1 = nn.LayerNorm(c.n_embd, eps=c.eps)
        self.attn = Attention(c)
        self.ln_2 = nn.LayerNorm(c.n_embd, eps=c.eps)
        self.mlp = MLP(c)

    def forward(self, x):
        x = x + self.attn(self.ln_1(x))
        return x + self.mlp(self.ln_2(x))

    def fp8_metas(self, device):
        metas = getattr(self, "_fp8_metas", None)
        if metas is None:
            from ..ops.fp8 import Fp8Meta
            metas = self._fp8_metas = tuple(Fp8Meta(device) for _ in range(4))
        return metas

    def fused_params(self):
        p = (self.ln_1.weight, self.ln_1.bias, self.attn.c_attn.weight, self.attn.c_attn.bias,
             self.attn.c_proj.weight, self.attn.c_proj.bias, self.ln_2.weight, self.ln_2.bias,
             self.mlp.c_fc.weight, self.mlp.c_fc.bias, self.mlp.c_proj.weight, self.mlp.c_proj.bias)
        shadows = tuple(OF.weight_bf16(w) for w in (p[2], p[4], p[8], p[10]))
        return p, shadows


class GPT2(nn.Module):
    def __init__(self, config: GPT2Config | None = None):
        super().__init__()
        c = self.config = config or GPT2Config()
        self.transformer = nn.ModuleDict(dict(
            wte=nn.Embedding(c.vocab_size, c.n_embd),
            wpe=nn.Embedding(c.block_size, c.n_embd),
            h=nn.ModuleList([Block(c) for _ in range(c.n_layer)]),
            ln_f=nn.LayerNorm(c.n_embd, eps=c.eps),
        ))
        self.lm_head = nn.Linear(c.n_embd, c.vocab_size, bias=False)
        self.lm_head.weight = self.transformer.wte.weight          # tied
        self.apply(self._init)
        for n, p in self.named_parameters():
            if n.endswith("c_proj.weight"):                          # GPT-2 residual-projection scaling
                nn.init.normal_(p, 0.0, 0.02 / math.sqrt(2 * c.n_layer))

    @staticmethod
    def _init(m):
        if isinstance(m, nn.Linear):
            nn.init.normal_(m.weight, 0.0, 0.02)
            if m.bias is not None:
                nn.init.zeros_(m.bias)
        elif isinstance(m, nn.Embedding):
            nn.init.normal_(m.weight, 0.0, 0.02)

    def awaits_params(self, idx, *args, **kwargs):
        """The fused GPU forward fetches every block's weight shadows through await_param (OF.weight_bf16), so a
        k-of-n DistributedDataParallel forward is checked before every block without the per-op ParamUseMode
        dispatch (a PS worker still uses ParamUseMode: its LayerNorm / bias parameters must have
        ARRIVED before use, which only the per-op hook guarantees)."""
        return bool(getattr(idx, "is_cuda", False))

    def ddp_tied_rows(self):
        """The tied token-embedding / LM-head weight: DistributedDataParallel all-reduces its dense (LM-head) gradient
        as soon as the head's backward has produced it and gathers the embedding's rows at the end (split_tied)."""
        return self.transformer.wte.weight if self.lm_head.weight is self.transformer.wte.weight else None

    def _row_tail(self):
        ref = self.__dict__.get("_pdnn_row_tail")
        ddp = ref() if ref is not None else None
        return ddp if ddp is not None and ddp._tail is self.transformer.wte.weight else None

    def num_params(self, non_embedding=True):
        n = sum(p.numel() for p in self.parameters())
        return n - self.transformer.wpe.weight.numel() if non_embedding else n

    def flops_per_token(self, T=None):
        """Training FLOPs per token (6N + attention 12*L*D*T, PaLM appendix B accounting)."""
        c = self.config
        T = T or c.block_size
        return 6 * self.num_params() + 12 * c.n_layer * c.n_embd * T

    def _t_weights(self):
        ws = self.__dict__.get("_pdnn_t_ws")
        if ws is None:
            ws = [self.transformer.wte.weight]
            for blk in self.transformer.h:
                ws += [blk.attn.c_attn.weight, blk.attn.c_proj.weight, blk.mlp.c_fc.weight, blk.mlp.c_proj.weight]
            self.__dict__["_pdnn_t_ws"] = ws
        return ws

    def forward(self, idx, targets=None):
        B, T = idx.shape
        c = self.config
        assert T <= c.block_size, f"sequence length {T} > block size {c.block_size}"
        if not idx.is_cuda:
            return self._forward_reference(idx, targets)
        tr = self.transformer
        wte, wpe = tr.wte.weight, tr.wpe.weight
        pf = tuning.get("wt_prefetch")
        if pf and targets is not None and torch.is_grad_enabled():
            # the data-gradient GEMMs' transposed weight copies, refreshed in one launch at forward start
            # (instead of ~50 small transposes inside the backward)
            from ..ops.fused_resnet import _side_stream
            OF.prefetch_weight_t(self._t_weights(), _side_stream(idx.device) if pf == 2 else None)
        wte_k, wpe_k = OF.weight_bf16(wte), OF.weight_bf16(wpe)
        # tied wte: with targets the fused LM head and the embedding both accumulate into its arena gradient
        hd = targets is not None and direct_grad(wte) is not None
        ddp = self._row_tail() if hd and torch.is_grad_enabled() else None
        if ddp is not None:
            # split under DistributedDataParallel: the head announces wte, the embedding's rows go through
            # ddp.reduce_sparse_rows (wte is not an autograd input of the embedding)
            x = TX.EmbeddingFn.apply(idx.reshape(-1).long().contiguous(), T, wte_k, wpe_k, None, wpe, False, (ddp, wte))
        else:
            x = TX.EmbeddingFn.apply(idx.reshape(-1).long().contiguous(), T, wte_k, wpe_k, wte, wpe, hd)
        for blk in tr.h:
            params, shadows = blk.fused_params()
            metas = blk.fp8_metas(x.device) if c.fp8 else None
            x = TX.GPT2BlockFn.apply(x, (B, T, c.n_head, c.eps, metas), shadows, *params)
        if targets is None:
            xf = TX.layer_norm(x, tr.ln_f.weight, tr.ln_f.bias, c.eps)
            return OF.linear(xf, wte).view(B, T, -1)
        return TX.LMHeadLossFn.apply(x, targets.reshape(-1).long().contiguous(), c.eps, wte_k, tr.ln_f.weight,
                                     tr.ln_f.bias, wte, hd, ddp is not None, torch.is_grad_enabled())

    def _forward_reference(self, idx, targets=None):
        B, T = idx.shape
        tr = self.transformer
        pos = torch.arange(T, device=idx.device)
        ddp = self._row_tail() if targets is not None and torch.is_grad_enabled() else None
        if ddp is not None:     # split tied embedding (see forward): the rows reach wte through the DDP tail
            x = _RowTailEmbedding.apply(idx, tr.wte.weight.detach(), tr.wpe(pos), (ddp, tr.wte.weight))
        else:
            x = tr.wte(idx) + tr.wpe(pos)
        for blk in tr.h:
            x = blk(x)
        logits = self.lm_head(tr.ln_f(x))
        if targets is None:
            return logits
        return F.cross_entropy(logits.float().view(-1, logits.shape[-1]), targets.reshape(-1))


class _RowTailEmbedding(torch.autograd.Function):
    """x = table[idx] + pos (reference path): the table is a detached view of the tied wte, so autograd's only edge
    into wte is the LM head's; the embedding rows reach wte.grad through DistributedDataParallel.reduce_sparse_rows
    in the backward.  ``pos`` [T][D] carries the autograd edge (its gradient is g summed over the batch); ``tail`` =
    (ddp, wte) is a tuple so that autograd adds no edge into wte (which would hold wte's AccumulateGrad -- and with it
    DDP's bucket 0 -- until this node has run)."""

    @staticmethod
    def forward(ctx, idx, table, pos, tail):
        ctx.save_for_backward(idx)
        ctx.ddp, ctx.wte = tail
        return F.embedding(idx, table) + pos

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        ddp, wte = ctx.ddp, ctx.wte
        ctx.ddp = ctx.wte = None
        gw = wte.grad
        ddp.reduce_sparse_rows(wte, idx, g, lambda i, r, sc: gw.index_add_(0, i, r.to(gw.dtype), alpha=sc))
        return None, None, g.sum(0), None


def build_gpt2(name: str = "gpt2_small", **kw) -> GPT2:
    base = CONFIGS[name.lower()]
    cfg = GPT2Config(**{**base.__dict__, **kw})
    return GPT2(cfg)
