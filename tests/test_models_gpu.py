"""End-to-end numerics of the fused GPU model paths against the CPU fp32 reference forward/backward of
the SAME module (identical weights): logits, loss, every parameter gradient, BN running statistics."""
import copy

import pytest
import torch

from bf16_mirror import cos, mirror, round_bf16

pytestmark = pytest.mark.gpu


def rel(a, b):
    """relative L2 error (see test_fused_blocks_gpu.rel for why not max-abs)."""
    a, b = a.float().cpu().flatten(), b.float().cpu().flatten()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def _run(model, x, y):
    from pytorch_distributed_nn_amd.ops import functional as OF
    model.zero_grad(set_to_none=True)
    out = model(x)
    loss = OF.cross_entropy(out, y)
    loss.backward()
    return out, loss


@pytest.mark.parametrize("name,shape,nc", [
    ("resnet50", (8, 3, 128, 128), 1000),
    ("ResNet18", (8, 3, 32, 32), 10),
    ("ResNet50", (8, 3, 32, 32), 10),
    ("LeNet", (8, 1, 28, 28), 10),
    ("mlp_cpp", (16, 784), 10),
])
def test_model_matches_cpu_reference(name, shape, nc):
    from pytorch_distributed_nn_amd.models import build_model
    torch.manual_seed(0)
    ref = build_model(name, nc)
    gpu = copy.deepcopy(ref).cuda()
    x = torch.randn(*shape)
    y = torch.randint(0, nc, (shape[0],))
    out_r, loss_r = _run(ref, x, y)
    out_g, loss_g = _run(gpu, x.cuda(), y.cuda())
    # deep bf16 networks: compare with a magnitude-relative bound and direction (cosine) of every grad
    # 16-50 bf16 BN/ReLU layers on an 8-image batch: per-block mask-flip noise compounds (see
    # test_fused_blocks_gpu for the tight per-block bounds)
    assert rel(out_g, out_r) < 3e-1, (name, rel(out_g, out_r))
    assert abs(loss_g.item() - loss_r.item()) < 3e-2 * max(1.0, abs(loss_r.item()))
    # Gradient DIRECTION is only a meaningful check where the quantity is well conditioned: in a random-init
    # ResNet-50 at batch 8 the reference itself is chaotic (rounding only the INPUT to bf16, everything else
    # fp32, moves the stem weight-gradient cosine to 0.47; ResNet-18: 0.98).  So: every gradient must exist
    # and be finite; shallow nets (LeNet, MLP) must match everywhere; deep nets at the classifier head.
    deep = name.lower().startswith("resnet")
    head = {"resnet50": "fc.", "ResNet18": "linear.", "ResNet50": "linear."}.get(name, "")
    for (n, pr), (_, pg) in zip(ref.named_parameters(), gpu.named_parameters()):
        assert pg.grad is not None, n
        assert torch.isfinite(pg.grad).all(), n
        if not deep or n.startswith(head):
            cos = torch.nn.functional.cosine_similarity(pg.grad.float().cpu().flatten(), pr.grad.flatten(), dim=0)
            assert cos > 0.97, (name, n, float(cos), rel(pg.grad, pr.grad))
    for (n, br), (_, bg) in zip(ref.named_buffers(), gpu.named_buffers()):
        if br.dtype.is_floating_point:
            assert rel(bg, br) < (1e-1 if deep else 3e-2), (name, n)
        else:
            assert torch.equal(bg.cpu(), br), (name, n)


def test_resnet50_train_step_flat_sgd():
    """A few fused-SGD steps on the flat arena reduce the loss on a fixed batch (memorisation)."""
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.optim import SGD, flatten_module
    from pytorch_distributed_nn_amd.ops import functional as OF
    torch.manual_seed(0)
    m = build_model("resnet50").cuda()
    flatten_module(m)
    opt = SGD(m.parameters(), lr=0.01, momentum=0.9)
    x = torch.randn(16, 3, 64, 64, device="cuda").to(torch.bfloat16)
    y = torch.randint(0, 1000, (16,), device="cuda")
    losses = []
    for _ in range(8):
        opt.zero_grad()
        loss = OF.cross_entropy(m(x), y)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert all(l == l for l in losses)
    assert losses[-1] < 0.6 * losses[0], losses


@pytest.mark.parametrize("arch", ["resnet50_small", "gpt2_tiny"])
def test_direct_grad_accumulation_matches_autograd_path(arch):
    """Fused ops accumulate flat-arena gradients in place (optim.flat.direct_grad): same gradients as the
    returned-gradient path, accumulation across two backwards, and every grad-ready hook fires once."""
    import copy
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.optim.flat import flatten_module, register_grad_ready_hook
    torch.manual_seed(0)
    if arch == "gpt2_tiny":
        m = build_model("gpt2_tiny").cuda()
        idx = torch.randint(0, 512, (2, 128), device="cuda")
        run = lambda net: net(idx, idx.roll(1, 1))
    else:
        m = build_model("resnet50").cuda()
        xin = torch.randn(4, 3, 64, 64, device="cuda")
        y = torch.randint(0, 1000, (4,), device="cuda")
        from pytorch_distributed_nn_amd.ops import functional as OF
        run = lambda net: OF.cross_entropy(net(xin), y)
    ref = copy.deepcopy(m)
    fp = flatten_module(m)
    counts = {}
    for p in fp.params:
        register_grad_ready_hook(p, lambda q: counts.__setitem__(id(q), counts.get(id(q), 0) + 1))
    fp.zero_grad()
    run(m).backward()
    run(ref).backward()
    assert all(counts.get(id(p), 0) == 1 for p in fp.params), "each grad-ready hook fires exactly once"
    for (n, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
        assert torch.allclose(p.grad, q.grad, rtol=1e-3, atol=1e-5 * q.grad.abs().max().item()), n
    g1 = fp.grad.clone()
    run(m).backward()                      # accumulates
    assert torch.allclose(fp.grad, 2 * g1, rtol=1e-3, atol=1e-6 * g1.abs().max().item())


@pytest.mark.parametrize("name,shape,nc", [
    ("ResNet18", (32, 3, 32, 32), 10),
    ("ResNet50", (32, 3, 32, 32), 10),
    ("resnet50", (32, 3, 64, 64), 1000),
])
def test_every_block_in_situ_against_mirrored_reference(name, shape, nc):
    """End-to-end at batch 32: the whole network runs fused on the GPU; every residual block is then
    replayed on the bf16-mirrored fp32 CPU reference with the block's OWN recorded input and output
    gradient from that run, and its parameter gradients and input gradient must match (<= 5% relative L2,
    cosine >= 0.998).  End-to-end gradient comparisons of a random-init deep ResNet are meaningless beyond
    the head: the fp32 reference itself moves its gradients by 13-18% (ResNet-18) and >100% (ResNet-50)
    under a 1e-3 relative input perturbation, so bf16 noise is amplified chaotically.  Replaying each block
    in situ checks every BN-backward / residual / dgrad term at its real position and shape in the net."""
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.ops import functional as OF
    torch.manual_seed(0)
    base = build_model(name, nc)
    gpu = copy.deepcopy(base).cuda()
    rec = []
    for blk in gpu._blocks():
        f = blk.forward_nhwc

        def wrapped(x, f=f, blk=blk):
            y = f(x)
            e = {"x": x.detach().clone(), "blk": blk}
            y.register_hook(lambda g, e=e: e.__setitem__("g", g.detach().clone()))
            rec.append(e)
            return y
        blk.forward_nhwc = wrapped
    x = torch.randn(*shape)
    y = torch.randint(0, nc, (shape[0],))
    loss = OF.cross_entropy(gpu(x.cuda()), y.cuda())
    loss.backward()
    ref_blocks = list(base._blocks())
    assert len(rec) == len(ref_blocks)
    worst = 0.0
    for i, (e, rb) in enumerate(zip(rec, ref_blocks)):
        ref = mirror(rb)
        xr = e["x"].float().cpu().permute(0, 3, 1, 2).contiguous().requires_grad_(True)
        yr = ref(xr)
        yr.backward(e["g"].float().cpu().permute(0, 3, 1, 2))
        for (n, pr), (_, pg) in zip(ref.named_parameters(), e["blk"].named_parameters()):
            r = rel(pg.grad, pr.grad)
            worst = max(worst, r)
            assert r < 5e-2 and cos(pg.grad, pr.grad) > 0.998, (name, i, n, r, cos(pg.grad, pr.grad))
        if i > 0:                       # this block's input gradient is the previous block's output gradient
            gin = rec[i - 1]["g"].float().cpu().permute(0, 3, 1, 2)
            assert rel(gin, xr.grad) < 5e-2 and cos(gin, xr.grad) > 0.998, (name, i, rel(gin, xr.grad))
    # the loss of the whole network against the mirrored reference (the logits of a 16-block random-init
    # ResNet-50 move by ~20% under bf16 noise, the mean loss by < 1%)
    from pytorch_distributed_nn_amd.ops import functional as OF2
    lr_ = OF2.cross_entropy(mirror(base)(round_bf16(x)), y).item()
    assert abs(loss.item() - lr_) / lr_ < 2e-2, (loss.item(), lr_)
