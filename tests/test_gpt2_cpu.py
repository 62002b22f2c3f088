"""GPT-2 model family on the CPU reference path: architecture, parameter count, tied head, training and
DDP over gloo (BASELINE.json config 4; the GPU path is checked against this in test_transformer_gpu.py)."""
import torch

from pytorch_distributed_nn_amd.models import build_model
from pytorch_distributed_nn_amd.models.gpt2 import GPT2Config, build_gpt2


def test_gpt2_small_shape_and_params():
    with torch.device("meta"):
        m = build_gpt2("gpt2_small")
    c = m.config
    assert (c.n_layer, c.n_head, c.n_embd, c.block_size, c.vocab_size) == (12, 12, 768, 1024, 50304)
    assert m.lm_head.weight is m.transformer.wte.weight
    n = sum(p.numel() for p in m.parameters())
    # 124.4M with the 50304-row padded vocabulary (GPT-2 small is 124M with 50257)
    assert 124_000_000 < n < 125_000_000
    assert m.flops_per_token(1024) > 6 * 85_000_000


def test_build_model_alias():
    m = build_model("GPT2-small")
    assert isinstance(m.config, GPT2Config) and m.config.n_layer == 12


def test_gpt2_tiny_trains_cpu():
    from pytorch_distributed_nn_amd.optim import AdamW
    torch.manual_seed(0)
    m = build_gpt2("gpt2_tiny")
    opt = AdamW(m.parameters(), lr=3e-3)
    idx = torch.randint(0, 64, (4, 65))
    x, y = idx[:, :-1], idx[:, 1:]
    losses = []
    for _ in range(25):
        opt.zero_grad()
        loss = m(x, y)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < 0.7 * losses[0]
    logits = m(x)
    assert logits.shape == (4, 64, m.config.vocab_size)
