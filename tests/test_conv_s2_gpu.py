"""Stride-2 3x3 halo kernels (csrc/kernels/conv_s2.hip) against fp32 torch: the forward (with BN statistics and the
BN + ReLU operand prologue) and the data gradient (every parity class in one launch, with the fused BN-backward
epilogue and the BN-backward operand prologue), at the ResNet stage-transition shapes and at odd half-resolution
sizes (tiles straddling image boundaries, partial last tiles)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
BF = torch.bfloat16

# (N, H, W, C, Ko) of the stride-2 conv's INPUT: ResNet-50 stages 2-4 at small batch, then odd half-resolution grids
SHAPES = [(2, 56, 56, 128, 128), (3, 28, 28, 256, 256), (5, 14, 14, 512, 512), (3, 18, 22, 128, 256),
          (2, 6, 10, 256, 128), (7, 2, 2, 128, 128), (1, 30, 8, 128, 384)]


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


def slab_close(a, b):
    C = a.shape[-1]
    ta, tb = a.view(-1, 2, C).double().sum(0), b.view(-1, 2, C).double().sum(0)
    assert torch.allclose(ta, tb, rtol=1e-5, atol=1e-5 * ta.abs().max().item() + 1e-6)


@pytest.fixture(scope="module")
def K():
    from pytorch_distributed_nn_amd.ops import kernels, _backend
    assert _backend.available()
    return kernels


@pytest.fixture(autouse=True)
def every_s2_route():
    """Route every direction through the stride-2 kernels (tuning s2_halo: 1 dgrad, 2 + 32 forward at any grid size,
    8 direct weight gradient, 16 dgrad operand prologue), whatever the measured defaults send where."""
    from pytorch_distributed_nn_amd import tuning
    old = tuning.set("s2_halo", 1 | 2 | 8 | 16 | 32)
    yield
    tuning.set("s2_halo", old)


def ref_fwd(x, w):
    return F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), None, 2, 1).permute(0, 2, 3, 1)


@pytest.mark.parametrize("shape", SHAPES)
def test_s2_forward_stats(K, shape):
    N, H, W, C, Ko = shape
    assert K.lib().pdnn_conv3x3s2_supported(N, H, W, C, Ko) == 1
    x = torch.randn(N, H, W, C, device="cuda").to(BF)
    w = (torch.randn(Ko, 3, 3, C, device="cuda") * 0.05).to(BF)
    y, slab = K.conv3x3s2(x, w, want_stats=True)
    ref = ref_fwd(x, w)
    assert y.shape == ref.shape
    assert rel(y, ref) < 1.5e-2
    yf = y.float().reshape(-1, Ko)
    s = slab.view(-1, 2, Ko).sum(0)
    assert torch.allclose(s[0], yf.sum(0), rtol=1e-3, atol=1e-2 * yf.abs().max().item())
    assert torch.allclose(s[1], (yf * yf).sum(0), rtol=1e-3, atol=1e-1)
    y2, _ = K.conv_fwd(x, w, 2, 1, want_stats=True)          # routed to the halo kernel
    assert torch.equal(y2, y)


@pytest.mark.parametrize("shape", SHAPES)
def test_s2_forward_prologue_matches_materialised(K, shape):
    N, H, W, C, Ko = shape
    t = torch.randn(N, H, W, C, device="cuda").to(BF)
    sc, sh = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.3
    a = K.bn_apply(t.view(-1, C), sc, sh, relu=True).view_as(t)
    w = (torch.randn(Ko, 3, 3, C, device="cuda") * 0.05).to(BF)
    y0, s0 = K.conv3x3s2(a, w, want_stats=True)
    y1, s1 = K.conv3x3s2(t, w, want_stats=True, pro=(sc, sh))
    assert torch.equal(y0, y1)
    slab_close(s0, s1)
    # the prologue's output written as a by-product (s2_halo bit 64): bitwise bn_apply's a1
    a_out = torch.full_like(t, float("nan"))
    y2, _ = K.conv3x3s2(t, w, want_stats=True, pro=(sc, sh), pro_out=a_out)
    assert torch.equal(y2, y0) and torch.equal(a_out, a)


def _dgrad_ref(w, dy, x_shape):
    N, H, W, C = x_shape
    x = torch.zeros(N, C, H, W, device="cuda", requires_grad=True)
    y = F.conv2d(x, w.float().permute(0, 3, 1, 2), None, 2, 1)
    y.backward(dy.float().permute(0, 3, 1, 2))
    return x.grad.permute(0, 2, 3, 1)


@pytest.mark.parametrize("shape", SHAPES)
def test_s2_dgrad_bn(K, shape):
    N, H, W, C, Ko = shape
    w = (torch.randn(Ko, 3, 3, C, device="cuda") * 0.05).to(BF)
    dy = torch.randn(N, H // 2, W // 2, Ko, device="cuda").to(BF)
    dx_ref = _dgrad_ref(w, dy, (N, H, W, C))
    dx = K.conv_dgrad(dy, w, (N, H, W, C), 2, 1)
    assert rel(dx, dx_ref) < 1.5e-2
    t = torch.randn(N, H, W, C, device="cuda").to(BF)
    mean, inv = torch.randn(C, device="cuda") * 0.1, torch.rand(C, device="cuda") + 0.5
    msc, msh = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.3
    gm, slab = K.conv_dgrad(dy, w, (N, H, W, C), 2, 1, bn=(t, mean, inv, msc, msh))
    z = t.float() * msc + msh
    gm_ref = dx_ref * (z > 0)
    far = z.abs() > 1e-3
    assert rel(gm[far], gm_ref[far]) < 1.5e-2
    s = slab.view(-1, 2, C).sum(0)
    gmf = gm.float().reshape(-1, C)
    xhat = ((t.float() - mean) * inv).reshape(-1, C)
    assert torch.allclose(s[0], gmf.sum(0), rtol=1e-3, atol=1e-3 * gmf.abs().sum(0).max().item())
    assert torch.allclose(s[1], (gmf * xhat).sum(0), rtol=1e-3, atol=1e-3 * (gmf * xhat).abs().sum(0).max().item())


@pytest.mark.parametrize("shape", SHAPES)
def test_s2_dgrad_pre_matches_separate_apply(K, shape):
    """dx = dgrad(bn_bwd_apply(gm, t)) with the apply in the halo staging: dt_out bitwise equal to the apply kernel,
    dx bitwise equal to the same kernel on that dt, with and without the fused BN-backward epilogue."""
    N, H, W, C, Ko = shape
    Ho, Wo = H // 2, W // 2
    w = (torch.randn(Ko, 3, 3, C, device="cuda") * 0.05).to(BF)
    gm = torch.randn(N, Ho, Wo, Ko, device="cuda").to(BF)
    t = torch.randn(N, Ho, Wo, Ko, device="cuda").to(BF)
    mean, inv = torch.randn(Ko, device="cuda") * 0.1, torch.rand(Ko, device="cuda") + 0.5
    g = torch.rand(Ko, device="cuda") + 0.5
    dg, db = torch.randn(Ko, device="cuda") * 50, torch.randn(Ko, device="cuda") * 50
    dt_ref = K.bn_bwd_apply(gm.view(-1, Ko), t.view(-1, Ko), mean, inv, g, dg, db, mode=0)[0].view_as(gm)
    assert K.dgrad_pre_ok(gm.shape, w.shape, 2, 1)
    dt_out = torch.empty_like(gm)
    dx = K.conv_dgrad(gm, w, (N, H, W, C), 2, 1, pre=(t, mean, inv, g, dg, db, dt_out))
    assert torch.equal(dt_out, dt_ref)
    assert torch.equal(dx, K.conv_dgrad(dt_ref, w, (N, H, W, C), 2, 1))
    t1 = torch.randn(N, H, W, C, device="cuda").to(BF)
    m1, i1 = torch.randn(C, device="cuda") * 0.1, torch.rand(C, device="cuda") + 0.5
    s1, h1 = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.3
    g1, sl1 = K.conv_dgrad(gm, w, (N, H, W, C), 2, 1, bn=(t1, m1, i1, s1, h1), pre=(t, mean, inv, g, dg, db, None))
    g1r, sl1r = K.conv_dgrad(dt_ref, w, (N, H, W, C), 2, 1, bn=(t1, m1, i1, s1, h1))
    assert torch.equal(g1, g1r)
    slab_close(sl1, sl1r)


def test_s2_off_switch_matches(K):
    """tuning s2_halo = 0 sends the same convs back to the implicit-GEMM engine: same results within bf16 rounding."""
    from pytorch_distributed_nn_amd import tuning
    N, H, W, C, Ko = 2, 28, 28, 256, 256
    x = torch.randn(N, H, W, C, device="cuda").to(BF)
    w = (torch.randn(Ko, 3, 3, C, device="cuda") * 0.05).to(BF)
    dy = torch.randn(N, H // 2, W // 2, Ko, device="cuda").to(BF)
    y1, _ = K.conv_fwd(x, w, 2, 1)
    d1 = K.conv_dgrad(dy, w, (N, H, W, C), 2, 1)
    old = tuning.set("s2_halo", 0)
    try:
        y0, _ = K.conv_fwd(x, w, 2, 1)
        d0 = K.conv_dgrad(dy, w, (N, H, W, C), 2, 1)
    finally:
        tuning.set("s2_halo", old)
    assert rel(y1, y0) < 1e-2 and rel(d1, d0) < 1e-2


@pytest.mark.parametrize("shape", [(2, 56, 56, 256), (3, 28, 28, 512), (2, 7, 9, 64), (1, 1, 1, 8)])
def test_subsample_matches_strided_view(K, shape):
    x = torch.randn(*shape, device="cuda").to(BF)
    assert torch.equal(K.subsample(x, 2), x[:, ::2, ::2, :].contiguous())


def test_shortcut_on_subsample_matches_strided_conv(K):
    """The stride-2 1x1 shortcut as a stride-1 conv of the subsampled input (tuning ds_sub): forward and weight
    gradient against the strided conv on the implicit-GEMM engine."""
    N, H, W, C, Ko = 4, 28, 28, 256, 512
    x = torch.randn(N, H, W, C, device="cuda").to(BF)
    w = (torch.randn(Ko, 1, 1, C, device="cuda") * 0.05).to(BF)
    xs = K.subsample(x, 2)
    y1, s1 = K.conv_fwd(xs, w, 1, 0, want_stats=True)
    y0, s0 = K.conv_fwd(x, w, 2, 0, want_stats=True)
    assert rel(y1, y0) < 1e-2
    dy = torch.randn(N, H // 2, W // 2, Ko, device="cuda").to(BF)
    d1 = K.conv_wgrad(xs, dy, 1, 1, 1, 0)
    d0 = K.conv_wgrad(x, dy, 1, 1, 2, 0)
    assert rel(d1, d0) < 5e-3


@pytest.mark.parametrize("shape", [(4, 56, 56, 128, 128), (3, 28, 28, 256, 256), (5, 14, 14, 512, 512),
                                   (3, 28, 56, 64, 192), (7, 6, 14, 128, 64)])
def test_s2_wgrad_direct(K, shape):
    """dW of a 3x3 / stride-2 / pad-1 conv on the parity-plane direct kernel against fp32 torch, accumulated (+=),
    with tiles straddling images and partial last tiles; and with the BN + ReLU prologue bitwise equal to the kernel on
    the materialised activation."""
    N, H, W, C, Ko = shape
    assert K.lib().pdnn_conv3x3s2_wgrad_supported(N, H, W, C, Ko) == 1
    x = torch.randn(N, H, W, C, device="cuda").to(BF)
    dy = torch.randn(N, H // 2, W // 2, Ko, device="cuda").to(BF)
    wr = torch.zeros(Ko, C, 3, 3, device="cuda", requires_grad=True)
    y = F.conv2d(x.float().permute(0, 3, 1, 2), wr, None, 2, 1)
    y.backward(dy.float().permute(0, 3, 1, 2))
    ref = wr.grad.permute(0, 2, 3, 1)
    base = torch.randn(Ko, 3, 3, C, device="cuda")
    out = K.conv_wgrad(x, dy, 3, 3, 2, 1, out=base.clone())
    assert rel(out - base, ref) < 5e-3
    sc, sh = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.3
    a = K.bn_apply(x.view(-1, C), sc, sh, relu=True).view_as(x)
    assert torch.equal(K.conv_wgrad(x, dy, 3, 3, 2, 1, pro=(sc, sh)), K.conv_wgrad(a, dy, 3, 3, 2, 1))


@pytest.mark.parametrize("shape", SHAPES)
def test_s2_dgrad_class_pairs_match_single_class(K, shape):
    """The class-pair data-gradient kernel (s2_halo bit 128: two parity classes per block) gives the single-class
    kernel's gm bitwise (same MFMA order per output) and its BN-backward sums up to atomic order."""
    from pytorch_distributed_nn_amd import tuning
    N, H, W, C, Ko = shape
    w = (torch.randn(Ko, 3, 3, C, device="cuda") * 0.05).to(BF)
    dy = torch.randn(N, H // 2, W // 2, Ko, device="cuda").to(BF)
    t = torch.randn(N, H, W, C, device="cuda").to(BF)
    mean, inv = torch.randn(C, device="cuda") * 0.1, torch.rand(C, device="cuda") + 0.5
    msc, msh = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.3
    g0, s0 = K.conv_dgrad(dy, w, (N, H, W, C), 2, 1, bn=(t, mean, inv, msc, msh))
    d0 = K.conv_dgrad(dy, w, (N, H, W, C), 2, 1)
    old = tuning.set("s2_halo", tuning.get("s2_halo") | 128)
    try:
        g1, s1 = K.conv_dgrad(dy, w, (N, H, W, C), 2, 1, bn=(t, mean, inv, msc, msh))
        d1 = K.conv_dgrad(dy, w, (N, H, W, C), 2, 1)
    finally:
        tuning.set("s2_halo", old)
    assert torch.equal(g1, g0) and torch.equal(d1, d0)
    slab_close(s1, s0)
