"""Each fused ResNet block (one autograd node = a hand-scheduled HIP kernel sequence) against the CPU
fp32 reference forward/backward of the same nn.Module that rounds to bf16 at the same points as the
kernels (tests/bf16_mirror.py): output, input gradient, every parameter gradient (<= 5% relative L2,
cosine >= 0.998) and the BN running statistics.  Shapes keep >= 256 elements per BN channel."""
import copy

import pytest
import torch

from bf16_mirror import mirror, round_bf16

pytestmark = pytest.mark.gpu


def rel(a, b):
    """relative L2 error.  Max-abs is the wrong metric through ReLU masks / max-pool argmax: a bf16 value
    rounding across 0 (or a tie) legitimately reroutes an O(1) gradient element."""
    a, b = a.float().cpu().flatten(), b.float().cpu().flatten()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def cos(a, b):
    return torch.nn.functional.cosine_similarity(a.float().cpu().flatten(), b.float().cpu().flatten(), dim=0).item()


def _check_block(block, x_nchw, tol_out=2e-2, tol_grad=5e-2):
    ref = mirror(block)
    gpu = copy.deepcopy(block).cuda()
    xr = round_bf16(x_nchw).detach().requires_grad_(True)
    yr = ref(xr)
    g = torch.randn_like(yr).to(torch.bfloat16).float()
    yr.backward(g)
    xg = x_nchw.permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16).requires_grad_(True)
    yg = gpu.forward_nhwc(xg)
    yg.backward(g.permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16))
    assert rel(yg, yr.permute(0, 2, 3, 1)) < tol_out
    assert rel(xg.grad, xr.grad.permute(0, 2, 3, 1)) < tol_grad
    assert cos(xg.grad, xr.grad.permute(0, 2, 3, 1)) > 0.998
    for (n, pr), (_, pg) in zip(ref.named_parameters(), gpu.named_parameters()):
        assert rel(pg.grad, pr.grad) < tol_grad, (n, rel(pg.grad, pr.grad))
        assert cos(pg.grad, pr.grad) > 0.998, (n, cos(pg.grad, pr.grad))
    for (n, br), (_, bg) in zip(ref.named_buffers(), gpu.named_buffers()):
        if br.dtype.is_floating_point:
            assert rel(bg, br) < 2e-2, n


@pytest.mark.parametrize("inp,planes,stride", [(256, 64, 1), (64, 64, 1), (256, 128, 2), (128, 64, 2)])
def test_bottleneck(inp, planes, stride):
    from pytorch_distributed_nn_amd.models.resnet import Bottleneck
    torch.manual_seed(0)
    blk = Bottleneck(inp, planes, stride, "downsample")
    _check_block(blk, torch.randn(8, inp, 16, 16))


@pytest.mark.parametrize("inp,planes,stride", [(64, 64, 1), (64, 128, 2)])
def test_basic_block(inp, planes, stride):
    from pytorch_distributed_nn_amd.models.resnet import BasicBlock
    torch.manual_seed(0)
    blk = BasicBlock(inp, planes, stride, "shortcut")
    _check_block(blk, torch.randn(8, inp, 16, 16))


@pytest.mark.parametrize("imagenet", [True, False])
def test_stem(imagenet):
    import torch.nn as nn
    import torch.nn.functional as F
    from pytorch_distributed_nn_amd.ops import functional as OF
    from pytorch_distributed_nn_amd.ops.fused_resnet import StemFn, stem_shadow
    torch.manual_seed(0)
    k, st, pad = (7, 2, 3) if imagenet else (3, 1, 1)
    conv = nn.Conv2d(3, 64, k, st, pad, bias=False)
    bn = nn.BatchNorm2d(64)
    conv_g, bn_g = copy.deepcopy(conv).cuda(), copy.deepcopy(bn).cuda()   # before the reference step
    x = torch.randn(4, 3, 32, 32)
    y = F.relu(bn(conv(x)))
    if imagenet:
        y = F.max_pool2d(y, 3, 2, 1)
    g = torch.randn_like(y)
    y.backward(g)
    xin = OF.nchw_to_nhwc_input(x.cuda())
    assert xin.shape == (4, 32, 32, 8)
    assert rel(xin[..., :3], x.permute(0, 2, 3, 1)) < 1e-2 and xin[..., 3:].abs().max() == 0
    yg = StemFn.apply(xin, (st, pad, imagenet, True, 0.1, 1e-5), [bn_g.running_mean, bn_g.running_var],
                      [stem_shadow(conv_g.weight, 8)], conv_g.weight, bn_g.weight, bn_g.bias)
    yg.backward(g.permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16))
    assert rel(yg, y.permute(0, 2, 3, 1)) < 3e-2
    assert rel(conv_g.weight.grad, conv.weight.grad) < 1.5e-1
    assert rel(bn_g.weight.grad, bn.weight.grad) < 1.5e-1
    assert rel(bn_g.bias.grad, bn.bias.grad) < 1.5e-1
    assert rel(bn_g.running_var, bn.running_var) < 2e-2


@pytest.mark.parametrize("flat", [True, False])
def test_side_stream_wgrad_matches_serial(monkeypatch, flat):
    """Weight gradients on the side stream (deferred join for arena gradients, immediate join for returned
    ones) == the serial schedule, for a whole ImageNet ResNet-50 at batch 4.  Two back-to-back backwards at
    the same weights with a zero_grad between them: the second one's zero-fill would race with the first
    one's side-stream atomics if the end-of-backward join did not hold."""
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.ops import functional as OF
    from pytorch_distributed_nn_amd.optim import SGD, flatten_module
    torch.manual_seed(0)
    m0 = build_model("resnet50", 1000)
    ms = [copy.deepcopy(m0).cuda() for _ in range(3)]
    opts = [None] * 3
    if flat:
        for m in ms:
            flatten_module(m)
        opts = [SGD(m.parameters(), lr=0.05, momentum=0.9) for m in ms]
    g = torch.Generator().manual_seed(1)
    data = [(torch.randn(4, 3, 96, 96, generator=g).cuda().to(torch.bfloat16), torch.randint(0, 1000, (4,), generator=g).cuda())
            for _ in range(2)]
    from pytorch_distributed_nn_amd import tuning
    grads = []
    for side, m, o in zip((1, 0, 0), ms, opts):
        old = tuning.set("side_wgrad", side)
        for x, y in data:
            if o is not None:
                o.zero_grad()
            else:
                m.zero_grad()
            OF.cross_entropy(m(x), y).backward()
        torch.cuda.synchronize()
        tuning.set("side_wgrad", old)
        grads.append(torch.cat([p.grad.float().flatten() for p in m.parameters()]))
    floor = rel(grads[2], grads[1])          # serial vs serial: fp32 atomics ordering
    r = rel(grads[0], grads[1])
    assert r < 10 * floor + 1e-3, (r, floor)
