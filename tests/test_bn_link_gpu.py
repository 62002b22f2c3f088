"""Hand-off between consecutive identity Bottlenecks (ops/fused_resnet.py _BnLink, tuning bn_link): the upper
block's conv1 data gradient (conv_dgrad ``bn_mask``, the C3_RESBN epilogue of the A-stationary 1x1 kernel)
also applies the lower block's output ReLU mask and reduces its BN3 backward sums.

* kernel: gm = (dy.W + res * res_mask) * bn_mask and the slab sums of gm, gm * xhat against fp32 torch;
* chain of Bottlenecks: every parameter / input gradient with the hand-off equal to the unlinked schedule
  (at the fp32 reduction-order floor), and the lower block's bn_bwd_reduce pass really skipped;
* a second consumer of a block output (its gradient is then a sum): the lower block detects it and falls
  back to its own masked reduction, still equal to the unlinked schedule."""
import copy

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def rel(a, b):
    a, b = a.float().flatten(), b.float().flatten()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


@pytest.fixture(scope="module")
def K():
    from pytorch_distributed_nn_amd.ops import kernels, _backend
    assert _backend.available()
    return kernels


def _bits(keep, C):
    b = (keep.view(-1, C // 8, 8).to(torch.int32) << torch.arange(8, device="cuda", dtype=torch.int32)).sum(-1)
    return b.to(torch.uint8).contiguous()


@pytest.mark.parametrize("shape", [(2, 56, 56, 64, 256), (3, 28, 28, 128, 512), (4, 14, 14, 128, 1024),
                                   (3, 9, 7, 64, 256), (1, 5, 3, 64, 64), (2, 7, 7, 128, 192)])
@pytest.mark.parametrize("with_res_mask", [True, False])
@pytest.mark.parametrize("with_pre", [False, True])
def test_conv_dgrad_resbn_epilogue(K, shape, with_res_mask, with_pre):
    N, H, W, Kc, C = shape
    P = N * H * W
    w = (torch.randn(Kc, 1, 1, C, device="cuda") * 0.1).to(BF)
    dy = torch.randn(N, H, W, Kc, device="cuda").to(BF)
    pre = None
    if with_pre:
        t0 = torch.randn(N, H, W, Kc, device="cuda").to(BF)
        m0, i0 = torch.randn(Kc, device="cuda") * 0.1, torch.rand(Kc, device="cuda") + 0.5
        g0 = torch.rand(Kc, device="cuda") + 0.5
        dg0, db0 = torch.randn(Kc, device="cuda") * 50, torch.randn(Kc, device="cuda") * 50
        pre = (t0, m0, i0, g0, dg0, db0, None)
        dt = K.bn_bwd_apply(dy.view(-1, Kc), t0.view(-1, Kc), m0, i0, g0, dg0, db0, mode=0)[0].view_as(dy)
    else:
        dt = dy
    assert K.resbn_ok(dy.shape, w.shape)
    res = torch.randn(N, H, W, C, device="cuda").to(BF)
    keep = torch.rand(P, C, device="cuda") > 0.5
    keep2 = torch.rand(P, C, device="cuda") > 0.3
    t = torch.randn(N, H, W, C, device="cuda").to(BF)
    mean, inv = torch.randn(C, device="cuda") * 0.1, torch.rand(C, device="cuda") + 0.5
    gm, slab = K.conv_dgrad(dy, w, (N, H, W, C), 1, 0, res=res, res_mask=_bits(keep, C) if with_res_mask else None,
                            bn=(t, mean, inv, None, None), bn_mask=_bits(keep2, C), pre=pre)
    dx = (dt.float().reshape(P, Kc) @ w.float().view(Kc, C))
    v = dx + res.float().view(P, C) * (keep if with_res_mask else 1)
    ref = v * keep2
    assert rel(gm.view(P, C), ref) < 1e-2
    assert (gm.view(P, C)[~keep2] == 0).all()
    gmf = gm.float().view(P, C)
    xhat = (t.float().view(P, C) - mean) * inv
    s = slab.view(-1, 2, C).sum(0)
    assert torch.allclose(s[0], gmf.sum(0), rtol=1e-3, atol=1e-3 * gmf.abs().sum(0).max().item())
    assert torch.allclose(s[1], (gmf * xhat).sum(0), rtol=1e-3, atol=1e-3 * (gmf * xhat).abs().sum(0).max().item())


def test_resbn_rejected_outside_areg_shapes(K):
    for k, c in ((512, 128), (256, 1024)):
        w = (torch.randn(k, 1, 1, c, device="cuda") * 0.1).to(BF)
        assert not K.resbn_ok((2, 8, 8, k), w.shape)


def _chain(planes=64, nblk=3):
    from pytorch_distributed_nn_amd.models.resnet import Bottleneck
    blocks = [Bottleneck(4 * planes, planes, 1, "downsample") for _ in range(nblk)]
    return torch.nn.ModuleList(blocks)


def _run(chain, x, g, bn_link, extra=False, count=None):
    from pytorch_distributed_nn_amd import tuning
    from pytorch_distributed_nn_amd.ops import kernels as Kmod
    old = tuning.set("bn_link", bn_link)   # default off (measured slower); the test forces both
    real = Kmod.bn_bwd_reduce
    calls = []

    def counting(*a, **k):
        calls.append(1)
        return real(*a, **k)
    Kmod.bn_bwd_reduce = counting
    try:
        xg = x.clone().requires_grad_(True)
        out, mids = xg, []
        for b in chain:
            out = b.forward_nhwc(out)
            mids.append(out)
        loss = (out.float() * g).sum()
        if extra:         # a second consumer of block 0's output: its gradient becomes a sum
            loss = loss + (mids[0].float() * g).sum() * 0.25
        loss.backward()
        torch.cuda.synchronize()
    finally:
        Kmod.bn_bwd_reduce = real
        tuning.set("bn_link", old)
    if count is not None:
        count.append(len(calls))
    return xg.grad, [p.grad.clone() for p in chain.parameters()]


@pytest.mark.parametrize("planes,hw", [(64, 28), (128, 14), (256, 7)])
@pytest.mark.parametrize("extra", [False, True])
def test_chain_gradients_equal_unlinked(planes, hw, extra):
    torch.manual_seed(0)
    base = _chain(planes)
    x = torch.randn(8, hw, hw, 4 * planes, device="cuda").to(BF)
    g = torch.randn(8, hw, hw, 4 * planes, device="cuda").to(BF).float()
    grads, counts = [], []
    for link in (0, 0, 1):
        m = copy.deepcopy(base).cuda().train()
        for p in m.parameters():
            p.grad = None
        grads.append(_run(m, x, g, link, extra=extra, count=counts))
    floor = max(rel(grads[1][0], grads[0][0]), 1e-4)
    assert rel(grads[2][0], grads[0][0]) < 20 * floor + 2e-3
    for a, b, c in zip(grads[0][1], grads[1][1], grads[2][1]):
        fl = max(rel(b, a), 1e-4)
        assert rel(c, a) < 20 * fl + 2e-3
    linked = planes in (64, 128)               # conv1 dgrad K = planes on the A-stationary kernel
    if linked and not extra:
        assert counts[2] == counts[0] - 2, counts    # blocks 0 and 1 reduced by the block above them
    elif linked:
        assert counts[2] == counts[0] - 1, counts    # block 0's gradient is a sum: it reduces itself
