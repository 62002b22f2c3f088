"""Long-reduction 1x1 / stride-1 conv kernel (csrc/kernels/conv1x1_wide.hip, K >= 512) against fp32 torch:
forward with BN statistics, data gradient plain / masked residual / fused BN backward, and the two operand
prologues -- BN-backward apply of an already-masked gradient (mode 0) and of the block output's gradient masked
by its ReLU bits (mode 3, the Bottleneck's conv3 data gradient) -- bitwise against apply-then-conv.  ResNet-50
shapes plus partial tiles."""
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
    N, H, W, C, Ko = shape            # forward: K input channels -> C outputs (here Kc = C_in, Ko = outputs)
    x = torch.randn(N, H, W, C, device="cuda").to(BF)
    w = (torch.randn(Ko, 1, 1, C, device="cuda") * 0.05).to(BF)
    assert K._panel_ok(N * H * W, C, Ko, 1, 1, 1, 0, fwd=True)
    y, slab = K.conv_fwd(x, w, 1, 0, want_stats=True)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2)).permute(0, 2, 3, 1)
    assert rel(y, ref) < 1.5e-2
    yf = y.float().reshape(-1, Ko)
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
    dx_ref = x.grad.permute(0, 2, 3, 1)
    assert K.dgrad_weight(dy.shape, w, (N, H, W, C), 1, 0) is not None     # routed to the transposed-weight kernel
    assert rel(K.conv_dgrad(dy, w, (N, H, W, C), 1, 0), dx_ref) < 1.5e-2
    res = torch.randn(N, H, W, C, device="cuda").to(BF)
    keep = torch.rand(N * H * W, C, device="cuda") > 0.5
    dxm = K.conv_dgrad(dy, w, (N, H, W, C), 1, 0, res=res, res_mask=_bits(keep))
    assert rel(dxm, dx_ref + res.float() * keep.view(N, H, W, C)) < 1.5e-2
    t = torch.randn(N, H, W, C, device="cuda").to(BF)
    mean, inv = torch.randn(C, device="cuda") * 0.1, torch.rand(C, device="cuda") + 0.5
    msc, msh = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.3
    gm, slab = K.conv_dgrad(dy, w, (N, H, W, C), 1, 0, bn=(t, mean, inv, msc, msh))
    z = t.float() * msc + msh
    far = z.abs() > 1e-3
    assert rel(gm[far], (dx_ref * (z > 0))[far]) < 1.5e-2
    s = slab.view(-1, 2, C).sum(0)
    gmf = gm.float().reshape(-1, C)
    xhat = ((t.float() - mean) * inv).reshape(-1, C)
    assert torch.allclose(s[0], gmf.sum(0), rtol=1e-3, atol=1e-3 * gmf.abs().sum(0).max().item())
    assert torch.allclose(s[1], (gmf * xhat).sum(0), rtol=1e-3, atol=1e-3 * (gmf * xhat).abs().sum(0).max().item())


def _pre(shape_nhwc):
    Kc = shape_nhwc[-1]
    g = torch.randn(*shape_nhwc, device="cuda").to(BF)
    t = torch.randn(*shape_nhwc, device="cuda").to(BF)
    mean, inv = torch.randn(Kc, device="cuda") * 0.1, torch.rand(Kc, device="cuda") + 0.5
    gamma = torch.rand(Kc, device="cuda") + 0.5
    dg, db = torch.randn(Kc, device="cuda") * 50, torch.randn(Kc, device="cuda") * 50
    return g, t, mean, inv, gamma, dg, db


@pytest.mark.parametrize("mode", [0, 3], ids=["gm-operand", "masked-gradient-operand"])
@pytest.mark.parametrize("shape", WIDE)
def test_wide_pre_matches_separate_apply(K, shape, mode):
    """dt = bn_bwd_apply(g, t) (mode 0: g already masked; mode 3: g masked by the ReLU bits) fused into the
    operand loads: dt_out bitwise equal to the apply kernel's output and the conv bitwise equal to the conv of
    that dt (same kernel), for the plain, masked-residual and fused-BN epilogues."""
    N, H, W, Kc, C = shape
    w = (torch.randn(Kc, 1, 1, C, device="cuda") * 0.05).to(BF)
    g, t, mean, inv, gamma, dg, db = _pre((N, H, W, Kc))
    bits = _bits(torch.rand(N * H * W, Kc, device="cuda") > 0.4) if mode == 3 else None
    dt_ref = K.bn_bwd_apply(g.view(-1, Kc), t.view(-1, Kc), mean, inv, gamma, dg, db, mode=mode,
                            msrc=bits)[0].view_as(g)
    assert K.dgrad_pre_ok(g.shape, w.shape, 1, 0)
    assert (mode == 3) <= K.dgrad_pre_mask_ok(g.shape, w.shape)
    dt_out = torch.empty_like(g)
    pre = (t, mean, inv, gamma, dg, db, dt_out) + ((bits,) if mode == 3 else ())
    dx = K.conv_dgrad(g, w, (N, H, W, C), 1, 0, pre=pre)
    assert torch.equal(dt_out, dt_ref)
    assert torch.equal(dx, K.conv_dgrad(dt_ref, w, (N, H, W, C), 1, 0))
    pre_n = (t, mean, inv, gamma, dg, db, None) + ((bits,) if mode == 3 else ())
    res = torch.randn(N, H, W, C, device="cuda").to(BF)
    rbits = _bits(torch.rand(N * H * W, C, device="cuda") > 0.5)
    dxr = K.conv_dgrad(g, w, (N, H, W, C), 1, 0, res=res, res_mask=rbits, pre=pre_n)
    assert torch.equal(dxr, K.conv_dgrad(dt_ref, w, (N, H, W, C), 1, 0, res=res, res_mask=rbits))
    t1 = torch.randn(N, H, W, C, device="cuda").to(BF)
    m1, i1 = torch.randn(C, device="cuda") * 0.1, torch.rand(C, device="cuda") + 0.5
    s1, h1 = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.3
    g1, sl1 = K.conv_dgrad(g, w, (N, H, W, C), 1, 0, bn=(t1, m1, i1, s1, h1), pre=pre_n)
    g1r, sl1r = K.conv_dgrad(dt_ref, w, (N, H, W, C), 1, 0, bn=(t1, m1, i1, s1, h1))
    assert torch.equal(g1, g1r) and torch.equal(sl1, sl1r)


def test_mask_operand_rejected_below_512(K):
    g, t, mean, inv, gamma, dg, db = _pre((2, 8, 8, 256))
    w = (torch.randn(256, 1, 1, 64, device="cuda") * 0.05).to(BF)
    bits = _bits(torch.rand(128, 256, device="cuda") > 0.5)
    assert not K.dgrad_pre_mask_ok(g.shape, w.shape)
    with pytest.raises(ValueError):
        K.conv_dgrad(g, w, (2, 8, 8, 64), 1, 0, pre=(t, mean, inv, gamma, dg, db, None, bits))
