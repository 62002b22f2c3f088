"""Multi-step training trajectories of the GPU path (bf16 HIP kernels, flat fp32 arena, fused SGD) against an
independent fp32 CPU reference (the same module and initial weights, stock torch autograd + torch.optim.SGD)
on a learnable synthetic task: the per-step losses must track each other, the loss must fall, and the final
weights must stay close.  Shallow, well-conditioned models only (LeNet, the reference MLPs, a CIFAR ResNet-18
at batch 128): for deep random-init nets at tiny batches the fp32 reference itself is chaotic
(test_models_gpu.py)."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.float().cpu().flatten(), b.float().cpu().flatten()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def _task(shape, nc, n_batches, seed=0):
    """Labels from a fixed random linear teacher of the input: a task the models can actually fit."""
    g = torch.Generator().manual_seed(seed)
    d = 1
    for s in shape[1:]:
        d *= s
    teacher = torch.randn(d, nc, generator=g)
    batches = []
    for _ in range(n_batches):
        x = torch.randn(*shape, generator=g)
        y = (x.reshape(shape[0], -1) @ teacher).argmax(1)
        batches.append((x, y))
    return batches


@pytest.mark.parametrize("name,shape,nc,steps,lr,tol,learns", [
    ("LeNet", (128, 1, 28, 28), 10, 30, 0.05, 0.05, True),
    ("mlp2", (128, 784), 10, 20, 0.1, 0.05, True),
    ("mlp_cpp", (128, 784), 10, 30, 0.5, 0.05, False),     # sigmoid stacks: slow on this task, track only
    ("mlp_s2", (128, 784), 10, 30, 0.5, 0.05, False),
    ("ResNet18", (128, 3, 32, 32), 10, 12, 0.02, 0.08, True),
])
def test_training_trajectory_tracks_fp32_cpu(name, shape, nc, steps, lr, tol, learns):
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.ops import functional as OF
    from pytorch_distributed_nn_amd.optim import SGD, flatten_module
    torch.manual_seed(0)
    ref = build_model(name, nc)
    gpu = copy.deepcopy(ref).cuda()
    flatten_module(gpu)
    opt_r = torch.optim.SGD(ref.parameters(), lr=lr, momentum=0.9)
    opt_g = SGD(gpu.parameters(), lr=lr, momentum=0.9)
    batches = _task(shape, nc, 4)
    lr_, lg_ = [], []
    for i in range(steps):
        x, y = batches[i % len(batches)]
        opt_r.zero_grad()
        loss_r = torch.nn.functional.cross_entropy(ref(x), y)
        loss_r.backward()
        opt_r.step()
        opt_g.zero_grad()
        loss_g = OF.cross_entropy(gpu(x.cuda()), y.cuda())
        loss_g.backward()
        opt_g.step()
        lr_.append(loss_r.item())
        lg_.append(loss_g.item())
    torch.cuda.synchronize()
    assert all(map(lambda v: v == v, lg_)), lg_
    # the task is learnt on both sides ...
    if learns:
        assert lr_[-1] < 0.8 * lr_[0] and lg_[-1] < 0.8 * lg_[0], (lr_, lg_)
    # ... along the same trajectory: every step's loss within tol of the fp32 reference (relative, or absolute
    # once the loss falls below 1)
    worst = max(abs(a - b) / max(abs(b), 1.0) for a, b in zip(lg_, lr_))
    assert worst < tol, (name, worst, lr_, lg_)
    wr = torch.cat([p.detach().flatten() for p in ref.parameters()])
    wg = torch.cat([p.detach().float().cpu().flatten() for p in gpu.parameters()])
    assert rel(wg, wr) < 2e-2, rel(wg, wr)


def _flagship(bn3_gain=0.1):
    """ImageNet-layout ResNet-50 with every residual branch's last BN gain at ``bn3_gain`` (the damped-branch form
    of the zero-init-residual recipe).  At gain 1 the random-init net's gradients are chaotic: a 1e-3 relative
    input perturbation moves the fp32 reference's own per-layer gradient cosine to 0.51-0.68 and stock torch bf16
    sits at -0.02-0.46 (the fused path alike), so no bf16 path can be checked against fp32 there; at 0.1 the
    perturbed fp32 cosine is >= 0.993 and bf16 paths sit at 0.95-0.98 (dev/probes/grad_cos.py, gpurun_out/r4_07)."""
    from pytorch_distributed_nn_amd.models import build_model
    torch.manual_seed(0)
    ref = build_model("resnet50").cuda()
    ref.fused = False                                      # plain torch ops, fp32, on the GPU
    with torch.no_grad():
        for n, p in ref.named_parameters():
            if n.endswith("bn3.weight"):
                p.fill_(bn3_gain)
    return ref


def test_flagship_resnet50_imagenet_trajectory_tracks_fp32():
    """the benchmarked model end to end -- ImageNet-layout ResNet-50 (7x7 stem, 1000-way head) at
    batch 64, 112x112 -- for 10 fused-SGD steps on the fused bf16 path (NCHW stem kernel, halo 3x3 convs and their
    direct weight gradients, A-stationary / long-reduction 1x1 kernels, fused BatchNorm passes, two HIP streams)
    against the same module run by stock torch in fp32 on the same GPU, same initial weights and batches.  The
    yardstick is stock torch's own mixed precision (autocast bf16, fp32 master weights) on the same trajectory:
    the fused path's loss and weight deviations from fp32 must be within 1.5x of autocast's (or under an absolute
    floor), and its weight updates must point the fp32 run's way."""
    from pytorch_distributed_nn_amd.ops import functional as OF
    from pytorch_distributed_nn_amd.optim import SGD, flatten_module
    ref = _flagship()
    fused = copy.deepcopy(ref)
    fused.fused = True
    flatten_module(fused)
    amp = copy.deepcopy(ref)
    w0 = torch.cat([p.detach().float().flatten() for p in ref.parameters()]).cpu()
    lr = 0.02
    opt_r = torch.optim.SGD(ref.parameters(), lr=lr, momentum=0.9, weight_decay=5e-5)
    opt_a = torch.optim.SGD(amp.parameters(), lr=lr, momentum=0.9, weight_decay=5e-5)
    opt_g = SGD(fused.parameters(), lr=lr, momentum=0.9, weight_decay=5e-5)
    batches = [(x.cuda(), y.cuda()) for x, y in _task((64, 3, 112, 112), 10, 3)]
    lr_, la_, lg_ = [], [], []
    for i in range(10):
        x, y = batches[i % len(batches)]
        opt_r.zero_grad()
        loss_r = torch.nn.functional.cross_entropy(ref(x), y)
        loss_r.backward()
        opt_r.step()
        opt_a.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss_a = torch.nn.functional.cross_entropy(amp(x).float(), y)
        loss_a.backward()
        opt_a.step()
        opt_g.zero_grad()
        loss_g = OF.cross_entropy(fused(x.to(torch.bfloat16)), y)
        loss_g.backward()
        opt_g.step()
        lr_.append(loss_r.item())
        la_.append(loss_a.item())
        lg_.append(loss_g.item())
    torch.cuda.synchronize()
    assert lr_[-1] < lr_[0] and lg_[-1] < lg_[0], (lr_, lg_)          # it trains
    dev = lambda ls: max(abs(a - b) / max(abs(b), 1.0) for a, b in zip(ls, lr_))     # noqa: E731
    assert dev(lg_) < max(0.02, 1.5 * dev(la_)), (dev(lg_), dev(la_), lr_, la_, lg_)
    flat = lambda m: torch.cat([p.detach().float().flatten() for p in m.parameters()]).cpu()   # noqa: E731
    wr, wa, wg = flat(ref), flat(amp), flat(fused)
    # deviation of the update (w - w0), where the precision differences live
    e_g, e_a = rel(wg - w0, wr - w0), rel(wa - w0, wr - w0)
    assert e_g < max(0.05, 1.5 * e_a), (e_g, e_a)
    cos = torch.nn.functional.cosine_similarity(wg - w0, wr - w0, dim=0).item()
    assert cos > 0.98, cos


def test_flagship_resnet50_first_step_gradients_per_tensor():
    """The flagship's first step, tensor by tensor (pins a single mis-routed layer that whole-model numbers would
    only show as drift): every parameter gradient of the fused bf16 path points the fp32 gradient's way (cosine
    > 0.9, norm within 10%), and on average as closely as stock torch autocast's does."""
    from pytorch_distributed_nn_amd.ops import functional as OF
    from pytorch_distributed_nn_amd.optim import flatten_module
    ref = _flagship()
    fused = copy.deepcopy(ref)
    fused.fused = True
    fp = flatten_module(fused)
    x, y = [t.cuda() for t in _task((64, 3, 112, 112), 10, 1)[0]]
    torch.nn.functional.cross_entropy(ref(x), y).backward()
    g_ref = [p.grad.float().flatten().clone() for p in ref.parameters()]
    ref.zero_grad()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        loss_a = torch.nn.functional.cross_entropy(ref(x).float(), y)
    loss_a.backward()
    g_amp = [p.grad.float().flatten().clone() for p in ref.parameters()]
    fp.zero_grad()
    OF.cross_entropy(fused(x.to(torch.bfloat16)), y).backward()
    torch.cuda.synchronize()
    bad, cs_g, cs_a = [], [], []
    for (n, _), pg, b, am in zip(ref.named_parameters(), fused.parameters(), g_ref, g_amp):
        a = pg.grad.float().flatten()
        cos = torch.nn.functional.cosine_similarity(a, b, dim=0).item()
        cs_g.append(cos)
        cs_a.append(torch.nn.functional.cosine_similarity(am, b, dim=0).item())
        ratio = (a.norm() / b.norm().clamp_min(1e-20)).item()
        if not (cos > 0.9 and 0.9 < ratio < 1.1):
            bad.append((n, round(cos, 4), round(ratio, 4)))
    assert not bad, bad
    mg, ma = sum(cs_g) / len(cs_g), sum(cs_a) / len(cs_a)
    assert mg > ma - 0.01, (mg, ma)


def test_flagship_resnet50_fp8_trajectory_tracks_fp32():
    """BASELINE config 5 numerics: the flagship with its stride-1 3x3 convs on the fp8 halo kernel (e4m3 forward,
    e5m2 data gradient, delayed per-tensor scales), 224x224 so stages 2 and 3 both run it, against the fp32 run of
    the same module: 8 fused-SGD steps whose losses and weight updates stay within fp8 precision of fp32 (2.5x
    autocast bf16's deviation or an absolute floor) and point the same way."""
    from pytorch_distributed_nn_amd.ops import functional as OF
    from pytorch_distributed_nn_amd.optim import SGD, flatten_module
    ref = _flagship()
    f8 = copy.deepcopy(ref)
    f8.fused = True
    f8.enable_fp8()
    flatten_module(f8)
    amp = copy.deepcopy(ref)
    w0 = torch.cat([p.detach().float().flatten() for p in ref.parameters()]).cpu()
    lr = 0.02
    opt_r = torch.optim.SGD(ref.parameters(), lr=lr, momentum=0.9, weight_decay=5e-5)
    opt_a = torch.optim.SGD(amp.parameters(), lr=lr, momentum=0.9, weight_decay=5e-5)
    opt_g = SGD(f8.parameters(), lr=lr, momentum=0.9, weight_decay=5e-5)
    batches = [(x.cuda(), y.cuda()) for x, y in _task((32, 3, 224, 224), 10, 2)]
    lr_, la_, lg_ = [], [], []
    for i in range(8):
        x, y = batches[i % len(batches)]
        opt_r.zero_grad()
        loss_r = torch.nn.functional.cross_entropy(ref(x), y)
        loss_r.backward()
        opt_r.step()
        opt_a.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss_a = torch.nn.functional.cross_entropy(amp(x).float(), y)
        loss_a.backward()
        opt_a.step()
        opt_g.zero_grad()
        loss_g = OF.cross_entropy(f8(x.to(torch.bfloat16)), y)
        loss_g.backward()
        opt_g.step()
        lr_.append(loss_r.item())
        la_.append(loss_a.item())
        lg_.append(loss_g.item())
    torch.cuda.synchronize()
    used = [b for b in f8._blocks() if getattr(b, "_fp8_state", None) is not None and b._fp8_state.fwd.primed]
    assert len(used) == 3 + 5, len(used)                 # stage 2 (28x28) and stage 3 (14x14) stride-1 blocks
    assert all(b._fp8_state.bwd.primed for b in used)
    assert lg_[-1] < lg_[0], lg_
    dev = lambda ls: max(abs(a - b) / max(abs(b), 1.0) for a, b in zip(ls, lr_))     # noqa: E731
    assert dev(lg_) < max(0.03, 2.5 * dev(la_)), (dev(lg_), dev(la_), lr_, la_, lg_)
    flat = lambda m: torch.cat([p.detach().float().flatten() for p in m.parameters()]).cpu()   # noqa: E731
    wr, wa, wg = flat(ref), flat(amp), flat(f8)
    e_g, e_a = rel(wg - w0, wr - w0), rel(wa - w0, wr - w0)
    assert e_g < max(0.1, 2.5 * e_a), (e_g, e_a)
    cos = torch.nn.functional.cosine_similarity(wg - w0, wr - w0, dim=0).item()
    assert cos > 0.95, cos
