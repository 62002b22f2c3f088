"""LDS-halo 3x3 / stride-1 conv kernel (csrc/kernels/conv3x3.hip) against fp32 torch: forward with BN
statistics, data gradient (tap-flipped weight) with the fused BN-backward epilogue and with a residual,
at the ResNet shapes, odd image sizes (tiles straddling image boundaries, partial last tile) and both
output-channel tiles."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def slab_close(a, b):
    """Two statistics slabs (STAT_BINS bins of fp32 atomic sums) hold the same totals up to summation order."""
    C = a.shape[-1]
    ta, tb = a.view(-1, 2, C).double().sum(0), b.view(-1, 2, C).double().sum(0)
    assert torch.allclose(ta, tb, rtol=1e-5, atol=1e-5 * ta.abs().max().item() + 1e-6)


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


@pytest.fixture(scope="module")
def K():
    from pytorch_distributed_nn_amd.ops import kernels, _backend
    assert _backend.available()
    return kernels


SHAPES = [(2, 56, 56, 64, 64), (2, 28, 28, 128, 128), (3, 14, 14, 256, 256), (5, 7, 7, 512, 512),
          (3, 9, 11, 64, 192), (2, 5, 6, 128, 64), (1, 16, 16, 192, 128), (7, 3, 3, 64, 128),
          (3, 7, 9, 64, 64), (5, 14, 14, 64, 64), (1, 1, 1, 64, 64)]


@pytest.fixture(params=[0, 1, 64, 128], ids=["nb-auto", "w64-resident", "nb64", "nb128"])
def nb(request, K):
    old = K.set_conv3x3_mode(1, request.param)
    oldf = K.lib().pdnn_conv3x3_force(1)        # narrow images too (the router sends W < 12 to the GEMM engine)
    yield request.param
    K.lib().pdnn_conv3x3_force(oldf)
    K.set_conv3x3_mode(*old)


def conv_ref(x, w):
    return F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), None, 1, 1).permute(0, 2, 3, 1)


@pytest.mark.parametrize("shape", SHAPES)
def test_conv3x3_fwd_stats(K, nb, shape):
    N, H, W, C, Ko = shape
    assert K.lib().pdnn_conv3x3_supported(N, H, W, C, Ko) == 1
    x = torch.randn(N, H, W, C, device="cuda").to(BF)
    w = (torch.randn(Ko, 3, 3, C, device="cuda") * 0.1).to(BF)
    y, slab = K.conv3x3(x, w, want_stats=True)
    ref = conv_ref(x, w)
    assert rel(y, ref) < 1.5e-2
    yf = y.float().reshape(-1, Ko)
    s = slab.view(-1, 2, Ko).sum(0)
    assert torch.allclose(s[0], yf.sum(0), rtol=1e-3, atol=1e-2 * yf.abs().max().item())
    assert torch.allclose(s[1], (yf * yf).sum(0), rtol=1e-3, atol=1e-1)
    # routed through conv_fwd as well
    y2, _ = K.conv_fwd(x, w, 1, 1, want_stats=True)
    assert torch.equal(y2, y)


@pytest.mark.parametrize("shape", SHAPES)
def test_conv3x3_dgrad_bn_and_res(K, nb, shape):
    N, H, W, C, Ko = shape
    x = torch.randn(N, C, H, W, device="cuda", requires_grad=True)
    w = (torch.randn(Ko, 3, 3, C, device="cuda") * 0.1).to(BF)
    y = F.conv2d(x, w.float().permute(0, 3, 1, 2), None, 1, 1)
    dy = torch.randn(*y.permute(0, 2, 3, 1).shape, device="cuda").to(BF)
    y.backward(dy.float().permute(0, 3, 1, 2))
    dx_ref = x.grad.permute(0, 2, 3, 1)
    assert rel(K.conv_dgrad(dy, w, (N, H, W, C), 1, 1), dx_ref) < 1.5e-2
    res = torch.randn(N, H, W, C, device="cuda").to(BF)
    assert rel(K.conv_dgrad(dy, w, (N, H, W, C), 1, 1, res=res), dx_ref + res.float()) < 1.5e-2
    # fused BN backward: gm = dx * [t*msc + msh > 0], sums of gm and gm*(t-mean)*inv
    t = torch.randn(N, H, W, C, device="cuda").to(BF)
    mean, inv = torch.randn(C, device="cuda") * 0.1, torch.rand(C, device="cuda") + 0.5
    msc, msh = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.3
    gm, slab = K.conv_dgrad(dy, w, (N, H, W, C), 1, 1, bn=(t, mean, inv, msc, msh))
    z = t.float() * msc + msh
    mask = z > 0
    gm_ref = dx_ref * mask
    far = z.abs() > 1e-3          # the kernel's fma and torch's mul+add may round a ~0 pre-activation apart
    assert rel(gm[far], gm_ref[far]) < 1.5e-2
    s = slab.view(-1, 2, C).sum(0)
    gmf = gm.float().reshape(-1, C)
    xhat = ((t.float() - mean) * inv).reshape(-1, C)
    assert torch.allclose(s[0], gmf.sum(0), rtol=1e-3, atol=1e-3 * gmf.abs().sum(0).max().item())
    assert torch.allclose(s[1], (gmf * xhat).sum(0), rtol=1e-3, atol=1e-3 * (gmf * xhat).abs().sum(0).max().item())


def test_conv3x3_matches_gemm_engine_bitwise_stats_layout(K):
    """The halo kernel and the implicit-GEMM engine agree on a ResNet-50 stage-1 layer (bs 8)."""
    x = torch.randn(8, 56, 56, 64, device="cuda").to(BF)
    w = (torch.randn(64, 3, 3, 64, device="cuda") * 0.05).to(BF)
    old = K.set_conv3x3_mode(0)
    y0, s0 = K.conv_fwd(x, w, 1, 1, want_stats=True)
    K.set_conv3x3_mode(1)
    y1, s1 = K.conv_fwd(x, w, 1, 1, want_stats=True)
    K.set_conv3x3_mode(*old)
    assert rel(y1, y0) < 1e-2
    torch.testing.assert_close(s1.view(-1, 2, 64).sum(0), s0.view(-1, 2, 64).sum(0), rtol=2e-3, atol=1.0)


# ------------------------------------------------------------------- 1x1 pixel-panel kernel (K in {64, 128})
PANEL = [(2, 56, 56, 64, 256), (3, 28, 28, 128, 512), (1, 7, 7, 128, 2048), (2, 9, 11, 64, 64), (5, 14, 14, 64, 1024),
         (1, 1, 3, 128, 128), (4, 14, 14, 256, 1024), (3, 9, 7, 256, 64), (1, 1, 1, 256, 128), (2, 28, 28, 256, 64)]


@pytest.mark.parametrize("shape", PANEL)
def test_conv1x1_panel_fwd_stats(K, shape):
    N, H, W, C, Ko = shape
    x = torch.randn(N, H, W, C, device="cuda").to(BF)
    w = (torch.randn(Ko, 1, 1, C, device="cuda") * 0.1).to(BF)
    y, slab = K.conv_fwd(x, w, 1, 0, want_stats=True)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2)).permute(0, 2, 3, 1)
    assert rel(y, ref) < 1.5e-2
    assert slab.shape[0] == 2 * K.STAT_BINS
    yf = y.float().reshape(-1, Ko)
    s = slab.view(-1, 2, Ko).sum(0)
    assert torch.allclose(s[0], yf.sum(0), rtol=1e-3, atol=1e-2 * yf.abs().max().item())
    assert torch.allclose(s[1], (yf * yf).sum(0), rtol=1e-3, atol=1e-1)


@pytest.mark.parametrize("shape", PANEL)
def test_conv1x1_panel_dgrad(K, shape):
    """dx = dy . W (K = dy channels in {64, 128}) plain / masked residual / fused BN backward."""
    N, H, W, Kc, C = shape            # dy has Kc channels, dx has C
    x = torch.randn(N, C, H, W, device="cuda", requires_grad=True)
    w = (torch.randn(Kc, 1, 1, C, device="cuda") * 0.1).to(BF)
    y = F.conv2d(x, w.float().permute(0, 3, 1, 2))
    dy = torch.randn(*y.permute(0, 2, 3, 1).shape, device="cuda").to(BF)
    y.backward(dy.float().permute(0, 3, 1, 2))
    dx_ref = x.grad.permute(0, 2, 3, 1)
    assert rel(K.conv_dgrad(dy, w, (N, H, W, C), 1, 0), dx_ref) < 1.5e-2
    res = torch.randn(N, H, W, C, device="cuda").to(BF)
    keep = torch.rand(N * H * W, C, device="cuda") > 0.5
    bits = (keep.view(-1, C // 8, 8).to(torch.int32) << torch.arange(8, device="cuda", dtype=torch.int32)).sum(-1)
    dxm = K.conv_dgrad(dy, w, (N, H, W, C), 1, 0, res=res, res_mask=bits.to(torch.uint8).contiguous())
    assert rel(dxm, dx_ref + res.float() * keep.view(N, H, W, C)) < 1.5e-2
    t = torch.randn(N, H, W, C, device="cuda").to(BF)
    mean, inv = torch.randn(C, device="cuda") * 0.1, torch.rand(C, device="cuda") + 0.5
    msc, msh = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.3
    gm, slab = K.conv_dgrad(dy, w, (N, H, W, C), 1, 0, bn=(t, mean, inv, msc, msh))
    z = t.float() * msc + msh
    mask = z > 0
    far = z.abs() > 1e-3          # the kernel's fma and torch's mul+add may round a ~0 pre-activation apart
    assert rel(gm[far], (dx_ref * mask)[far]) < 1.5e-2
    s = slab.view(-1, 2, C).sum(0)
    gmf = gm.float().reshape(-1, C)
    xhat = ((t.float() - mean) * inv).reshape(-1, C)
    assert torch.allclose(s[0], gmf.sum(0), rtol=1e-3, atol=1e-3 * gmf.abs().sum(0).max().item())
    assert torch.allclose(s[1], (gmf * xhat).sum(0), rtol=1e-3, atol=1e-3 * (gmf * xhat).abs().sum(0).max().item())


# ------------------------------------------- BN-backward apply fused into the operand loads (pre=)
def _pre_operands(shape_nhwc, gamma=True):
    Ko = shape_nhwc[-1]
    gm = torch.randn(*shape_nhwc, device="cuda").to(BF)
    t = torch.randn(*shape_nhwc, device="cuda").to(BF)
    mean, inv = torch.randn(Ko, device="cuda") * 0.1, torch.rand(Ko, device="cuda") + 0.5
    g = torch.rand(Ko, device="cuda") + 0.5 if gamma else None
    dg, db = torch.randn(Ko, device="cuda") * 50, torch.randn(Ko, device="cuda") * 50
    return gm, t, mean, inv, g, dg, db


@pytest.mark.parametrize("shape", SHAPES)
def test_conv3x3_dgrad_pre_matches_separate_apply(K, nb, shape):
    """dx = conv3x3_dgrad(bn_bwd_apply(gm, t)) with the apply in the halo loads: dt_out bitwise equal to the
    apply kernel's output, dx bitwise equal to the dgrad of that dt (same kernel and tile), for the plain,
    residual and fused-BN epilogues."""
    N, H, W, C, Ko = shape
    w = (torch.randn(Ko, 3, 3, C, device="cuda") * 0.1).to(BF)
    gm, t, mean, inv, g, dg, db = _pre_operands((N, H, W, Ko), gamma=(Ko % 128 == 0))
    dt_ref = K.bn_bwd_apply(gm.view(-1, Ko), t.view(-1, Ko), mean, inv, g, dg, db, mode=0)[0].view_as(gm)
    assert K.dgrad_pre_ok(gm.shape, w.shape, 1, 1)
    exact = nb != 1          # nb=1: the plain dgrad runs the weight-resident kernel, pre= the streaming one
    chk = (lambda a, b: torch.equal(a, b)) if exact else (lambda a, b: rel(a, b) < 1e-2)
    dt_out = torch.empty_like(gm)
    dx = K.conv_dgrad(gm, w, (N, H, W, C), 1, 1, pre=(t, mean, inv, g, dg, db, dt_out))
    assert torch.equal(dt_out, dt_ref)
    assert chk(dx, K.conv_dgrad(dt_ref, w, (N, H, W, C), 1, 1))
    res = torch.randn(N, H, W, C, device="cuda").to(BF)
    keep = torch.rand(N * H * W, C, device="cuda") > 0.5
    bits = (keep.view(-1, C // 8, 8).to(torch.int32) << torch.arange(8, device="cuda", dtype=torch.int32)).sum(-1)
    bits = bits.to(torch.uint8).contiguous()
    dxr = K.conv_dgrad(gm, w, (N, H, W, C), 1, 1, res=res, res_mask=bits, pre=(t, mean, inv, g, dg, db, None))
    assert chk(dxr, K.conv_dgrad(dt_ref, w, (N, H, W, C), 1, 1, res=res, res_mask=bits))
    t1 = torch.randn(N, H, W, C, device="cuda").to(BF)
    m1, i1 = torch.randn(C, device="cuda") * 0.1, torch.rand(C, device="cuda") + 0.5
    s1, h1 = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.3
    g1, sl1 = K.conv_dgrad(gm, w, (N, H, W, C), 1, 1, bn=(t1, m1, i1, s1, h1), pre=(t, mean, inv, g, dg, db, None))
    g1r, sl1r = K.conv_dgrad(dt_ref, w, (N, H, W, C), 1, 1, bn=(t1, m1, i1, s1, h1))
    assert chk(g1, g1r)
    if exact:       # statistics bins are fp32 atomic sums: equal up to the summation order
        slab_close(sl1, sl1r)


@pytest.mark.parametrize("shape", PANEL)
def test_conv1x1_panel_pre_matches_separate_apply(K, shape):
    """The panel kernel's operand prologue (K in {64, 128}): same bits as apply-then-conv."""
    N, H, W, Kc, C = shape
    w = (torch.randn(Kc, 1, 1, C, device="cuda") * 0.1).to(BF)
    gm, t, mean, inv, g, dg, db = _pre_operands((N, H, W, Kc))
    dt_ref = K.bn_bwd_apply(gm.view(-1, Kc), t.view(-1, Kc), mean, inv, g, dg, db, mode=0)[0]
    wt = K.transpose_bf16(w.view(Kc, C))
    dt_out = torch.empty_like(gm)
    y, _ = K.conv1x1_panel(gm.view(-1, Kc), wt, pre=(t, mean, inv, g, dg, db, dt_out))
    y_ref, _ = K.conv1x1_panel(dt_ref, wt)
    assert torch.equal(dt_out.view(-1, Kc), dt_ref)
    assert torch.equal(y, y_ref)
    res = torch.randn(N * H * W, C, device="cuda").to(BF)
    yr, _ = K.conv1x1_panel(gm.view(-1, Kc), wt, res=res, pre=(t, mean, inv, g, dg, db, None))
    assert torch.equal(yr, K.conv1x1_panel(dt_ref, wt, res=res)[0])
    if Kc in (64, 256):       # routed through conv_dgrad (the K = 64 / 256 panel data gradient)
        assert K.dgrad_pre_ok(gm.shape, w.shape, 1, 0)
        dx = K.conv_dgrad(gm, w, (N, H, W, C), 1, 0, pre=(t, mean, inv, g, dg, db, None))
        assert torch.equal(dx.view(-1, C), y_ref)


def test_dgrad_pre_rejected_on_gemm_engine(K):
    # K = 192: neither the panel / A-stationary kernels (K <= 256 powers of two) nor the long-reduction one
    gm, t, mean, inv, g, dg, db = _pre_operands((2, 8, 8, 192))
    w = (torch.randn(192, 1, 1, 64, device="cuda") * 0.1).to(BF)
    assert not K.dgrad_pre_ok(gm.shape, w.shape, 1, 0)
    with pytest.raises(ValueError):
        K.conv_dgrad(gm, w, (2, 8, 8, 64), 1, 0, pre=(t, mean, inv, g, dg, db, None))


# ------------------------------------------- direct 3x3 weight gradient (conv3x3_wgrad.hip)
WGRAD3 = [(4, 56, 56, 64, 64), (2, 28, 28, 128, 128), (3, 14, 14, 256, 256), (5, 7, 7, 512, 512), (3, 9, 56, 64, 192),
          (2, 5, 14, 128, 64), (7, 3, 7, 64, 128), (1, 4, 7, 64, 64), (2, 13, 28, 192, 64)]


@pytest.mark.parametrize("shape", WGRAD3)
def test_conv3x3_wgrad_direct(K, shape):
    """dW of a 3x3 / stride-1 / pad-1 conv on the direct halo kernel against fp32 torch, accumulated into an
    existing gradient (+=), including tiles straddling image boundaries and partial last tiles."""
    N, H, W, C, Ko = shape
    assert K.lib().pdnn_conv3x3_wgrad_supported(N, H, W, C, Ko) == 1
    x = torch.randn(N, H, W, C, device="cuda").to(BF)
    dy = torch.randn(N, H, W, Ko, device="cuda").to(BF)
    wr = torch.zeros(Ko, C, 3, 3, device="cuda", requires_grad=True)
    y = F.conv2d(x.float().permute(0, 3, 1, 2), wr, None, 1, 1)
    y.backward(dy.float().permute(0, 3, 1, 2))
    ref = wr.grad.permute(0, 2, 3, 1)                      # [Ko][3][3][C]
    base = torch.randn(Ko, 3, 3, C, device="cuda")
    out = K.conv_wgrad(x, dy, 3, 3, 1, 1, out=base.clone())          # accumulates into out
    assert rel(out - base, ref) < 5e-3


# ------------------------------------------- BN + ReLU of the layer below applied while staging (pro=)
@pytest.mark.parametrize("shape", [(2, 56, 56, 64, 64), (2, 28, 28, 128, 128), (3, 14, 14, 256, 256),
                                   (3, 13, 14, 128, 64)])
def test_conv3x3_forward_prologue_matches_materialised(K, shape):
    """The halo forward and the direct weight gradient with the operand relu(t * sc + sh) formed while staging: bitwise
    equal to running them on bn_apply's materialised activation (same kernels, same tiles, bn_apply's rounding)."""
    N, H, W, C, Ko = shape
    t = torch.randn(N, H, W, C, device="cuda").to(BF)
    sc, sh = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.3
    a = K.bn_apply(t.view(-1, C), sc, sh, relu=True).view_as(t)
    w = (torch.randn(Ko, 3, 3, C, device="cuda") * 0.1).to(BF)
    y0, s0 = K.conv3x3(a, w, want_stats=True)
    y1, s1 = K.conv3x3(t, w, want_stats=True, pro=(sc, sh))
    assert torch.equal(y0, y1)
    slab_close(s0, s1)
    y2, _ = K.conv_fwd(t, w, 1, 1, pro=(sc, sh))          # routed to the halo kernel with the prologue
    assert torch.equal(y2, y0)
    assert K.conv3x3_pro_ok(tuple(t.shape), Ko)
    dy = torch.randn(N, H, W, Ko, device="cuda").to(BF)
    d0 = K.conv_wgrad(a, dy, 3, 3, 1, 1)
    d1 = K.conv_wgrad(t, dy, 3, 3, 1, 1, pro=(sc, sh))
    assert torch.equal(d0, d1)


@pytest.mark.parametrize("shape", [(2, 56, 56, 64, 256), (3, 28, 28, 128, 512), (2, 14, 14, 256, 1024), (1, 9, 7, 64, 64)])
def test_conv1x1_forward_prologue_matches_materialised(K, shape):
    """The A-stationary 1x1 forward with relu(t * sc + sh) applied to its activation fragments as they load (a
    Bottleneck conv3 reading t2 instead of a materialised a2): output bitwise equal to the same kernel on bn_apply's
    activation, statistics equal up to summation order; the weight gradient with the same prologue on the
    implicit-GEMM engine matches the one on the activation."""
    N, H, W, C, Ko = shape
    t = torch.randn(N, H, W, C, device="cuda").to(BF)
    sc, sh = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.3
    a = K.bn_apply(t.view(-1, C), sc, sh, relu=True).view_as(t)
    w = (torch.randn(Ko, 1, 1, C, device="cuda") * 0.1).to(BF)
    assert K.conv1x1_pro_ok(tuple(t.shape), Ko)
    y0, s0 = K.conv_fwd(a, w, 1, 0, want_stats=True)
    y1, s1 = K.conv_fwd(t, w, 1, 0, pro=(sc, sh), want_stats=True)
    assert torch.equal(y0, y1)
    slab_close(s0, s1)
    dy = torch.randn(N, H, W, Ko, device="cuda").to(BF)
    d0 = K.conv_wgrad(a, dy, 1, 1, 1, 0)
    d1 = K.conv_wgrad(t, dy, 1, 1, 1, 0, pro=(sc, sh))
    assert rel(d1, d0) < 1e-3
