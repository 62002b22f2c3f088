"""Long-reduction 1x1 / stride-1 conv kernel (csrc/kernels/conv1x1_wide.hip, K >= 512) against fp32 torch:
forward with BN statistics, data gradient plain / masked residual / fused BN backward, and the BN-backward apply
operand prologue bitwise against apply-then-conv.  The kernel is called directly (conv1x1_panel with K >= 512) at
ResNet-50 shapes plus partial tiles; conv_dgrad routes to it for K >= 512 with >= 1024 outputs (checked too)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
BF = torch.bfloat16

# (N, H, W, K = reduction channels, C = output channels)
WIDE = [(2, 28, 28, 512, 128), (3, 14, 14, 1024, 256), (5, 7, 7, 2048, 512), (4, 7, 7, 512, 2048),
        (2, 14, 14, 512, 1024), (3, 5, 7, 512, 64), (1, 1, 1, 1024, 64), (2, 9, 9, 768, 192)]


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


@pytest.fixture(scope="module")
def K():
    from pytorch_distributed_nn_amd.ops import kernels, _backend
    assert _backend.available()
    return kernels


def _bits(keep):
    P, C = keep.shape
    b = (keep.view(P, C // 8, 8).to(torch.int32) << torch.arange(8, device="cuda", dtype=torch.int32)).sum(-1)
    return b.to(torch.uint8).contiguous()


@pytest.mark.parametrize("shape", WIDE)
def test_wide_fwd_stats(K, shape):
    N, H, W, C, Ko = shape                    # y[P][Ko] = x[P][C] . w[Ko][C]^T, C >= 512
    x = torch.randn(N, H, W, C, device="cuda").to(BF)
    w = (torch.randn(Ko, C, device="cuda") * 0.05).to(BF)
    y, slab = K.conv1x1_panel(x.view(-1, C), w, want_stats=True)
    ref = x.float().view(-1, C) @ w.float().t()
    assert rel(y, ref) < 1.5e-2
    yf = y.float()
    s = slab.view(-1, 2, Ko).sum(0)
    assert torch.allclose(s[0], yf.sum(0), rtol=1e-3, atol=1e-2 * yf.abs().max().item())
    assert torch.allclose(s[1], (yf * yf).sum(0), rtol=1e-3, atol=1e-1)


@pytest.mark.parametrize("shape", WIDE)
def test_wide_dgrad_epilogues(K, shape):
    N, H, W, Kc, C = shape            # dy has Kc channels, dx has C
    x = torch.randn(N, C, H, W, device="cuda", requires_grad=True)
    w = (torch.randn(Kc, 1, 1, C, device="cuda") * 0.05).to(BF)
    y = F.conv2d(x, w.float().permute(0, 3, 1, 2))
    dy = torch.randn(*y.permute(0, 2, 3, 1).shape, device="cuda").to(BF)
    y.backward(dy.float().permute(0, 3, 1, 2))
    dx_ref = x.grad.permute(0, 2, 3, 1).reshape(-1, C)
    wt = K.transpose_bf16(w.view(Kc, C))
    d2 = dy.view(-1, Kc)
    assert rel(K.conv1x1_panel(d2, wt)[0], dx_ref) < 1.5e-2
    # routed there by conv_dgrad for the stage-4 conv1 shapes (K >= 512, >= 1024 outputs)
    if C >= 1024:
        assert K.dgrad_weight(dy.shape, w, (N, H, W, C), 1, 0) is not None
        assert torch.equal(K.conv_dgrad(dy, w, (N, H, W, C), 1, 0).view(-1, C), K.conv1x1_panel(d2, wt)[0])
    res = torch.randn(N * H * W, C, device="cuda").to(BF)
    keep = torch.rand(N * H * W, C, device="cuda") > 0.5
    dxm, _ = K.conv1x1_panel(d2, wt, res=res, res_mask=_bits(keep))
    assert rel(dxm, dx_ref + res.float() * keep) < 1.5e-2
    t = torch.randn(N * H * W, C, device="cuda").to(BF)
    mean, inv = torch.randn(C, device="cuda") * 0.1, torch.rand(C, device="cuda") + 0.5
    msc, msh = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.3
    gm, slab = K.conv1x1_panel(d2, wt, bn=(t, mean, inv, msc, msh))
    z = t.float() * msc + msh
    far = z.abs() > 1e-3
    assert rel(gm[far], (dx_ref * (z > 0))[far]) < 1.5e-2
    s = slab.view(-1, 2, C).sum(0)
    gmf = gm.float()
    xhat = (t.float() - mean) * inv
    assert torch.allclose(s[0], gmf.sum(0), rtol=1e-3, atol=1e-3 * gmf.abs().sum(0).max().item())
    assert torch.allclose(s[1], (gmf * xhat).sum(0), rtol=1e-3, atol=1e-3 * (gmf * xhat).abs().sum(0).max().item())


@pytest.mark.parametrize("shape", WIDE)
def test_wide_pre_matches_separate_apply(K, shape):
    """dt = bn_bwd_apply(gm, t) fused into the operand loads: dt_out bitwise equal to the apply kernel's output
    and the conv bitwise equal to the conv of that dt (same kernel), plain and masked-residual epilogues."""
    N, H, W, Kc, C = shape
    P = N * H * W
    w = (torch.randn(Kc, C, device="cuda") * 0.05).to(BF)
    wt = K.transpose_bf16(w)
    g = torch.randn(P, Kc, device="cuda").to(BF)
    t = torch.randn(P, Kc, device="cuda").to(BF)
    mean, inv = torch.randn(Kc, device="cuda") * 0.1, torch.rand(Kc, device="cuda") + 0.5
    gamma = torch.rand(Kc, device="cuda") + 0.5
    dg, db = torch.randn(Kc, device="cuda") * 50, torch.randn(Kc, device="cuda") * 50
    dt_ref = K.bn_bwd_apply(g, t, mean, inv, gamma, dg, db, mode=0)[0]
    dt_out = torch.empty_like(g)
    y, _ = K.conv1x1_panel(g, wt, pre=(t, mean, inv, gamma, dg, db, dt_out))
    assert torch.equal(dt_out, dt_ref)
    assert torch.equal(y, K.conv1x1_panel(dt_ref, wt)[0])
    res = torch.randn(P, C, device="cuda").to(BF)
    rbits = _bits(torch.rand(P, C, device="cuda") > 0.5)
    yr, _ = K.conv1x1_panel(g, wt, res=res, res_mask=rbits, pre=(t, mean, inv, gamma, dg, db, None))
    assert torch.equal(yr, K.conv1x1_panel(dt_ref, wt, res=res, res_mask=rbits)[0])
