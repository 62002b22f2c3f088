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


def _split_tied(rank, world, split):
    """One GPT-2 step under DDP over gloo: the tied wte/LM-head gradient, the bucket plan, the per-bucket launch order."""
    import torch.distributed as dist
    from pytorch_distributed_nn_amd.parallel.ddp import DistributedDataParallel
    torch.manual_seed(5)
    m = build_gpt2("gpt2_tiny")
    ddp = DistributedDataParallel(m, bucket_cap_mb=0.25, split_tied=split)
    g = torch.Generator().manual_seed(11)
    idx = torch.randint(0, 512, (2 * world, 33), generator=g)
    x, y = idx[rank * 2:(rank + 1) * 2, :-1], idx[rank * 2:(rank + 1) * 2, 1:]
    ddp.zero_grad()
    ddp(x, y).backward()
    wte = m.transformer.wte.weight
    out = {"wte": wte.grad.clone(), "wpe": m.transformer.wpe.weight.grad.clone(),
           "h0": m.transformer.h[0].attn.c_attn.weight.grad.clone(), "split": ddp._tail is not None,
           "bucket0": ddp._pbucket[id(wte)], "nb": len(ddp.buckets), "order": list(ddp.last_launch_order)}
    if rank == 0:         # single-process reference on the global batch, same init
        torch.manual_seed(5)
        ref = build_gpt2("gpt2_tiny")
        ref(idx[:, :-1], idx[:, 1:]).backward()
        out["ref_wte"] = ref.transformer.wte.weight.grad.clone()
        out["ref_wpe"] = ref.transformer.wpe.weight.grad.clone()
    dist.barrier()
    return out


def test_ddp_split_tied_embedding_equals_averaged_tied_gradient():
    """VERDICT r5 #2a: the tied wte's dense LM-head part is bucket 0 (launched first, right after the head's backward),
    the embedding rows are gathered and added after it -- the result equals the averaged tied gradient of the
    single-process global batch, and equals the unsplit DDP path."""
    from dist_utils import run_world
    res = run_world(_split_tied, 2, (True,))
    base = run_world(_split_tied, 2, (False,))
    r0 = res[0]
    assert r0["split"] and not base[0]["split"]
    assert r0["bucket0"] == 0 and r0["order"][0] == 0          # the wte bucket goes out first
    assert base[0]["bucket0"] == base[0]["nb"] - 1              # unsplit: reverse order puts it last
    for r in res + base:
        torch.testing.assert_close(r["wte"], r0["ref_wte"], rtol=1e-4, atol=1e-6)
        torch.testing.assert_close(r["wpe"], r0["ref_wpe"], rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(res[0]["h0"], base[0]["h0"], rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(res[1]["wte"], res[0]["wte"], rtol=0, atol=0)
