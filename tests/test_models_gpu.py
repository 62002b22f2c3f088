"""End-to-end numerics of the fused GPU model paths against the CPU fp32 reference forward/backward of
the SAME module (identical weights): logits, loss, every parameter gradient, BN running statistics."""
import copy

import pytest
import torch

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
