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
