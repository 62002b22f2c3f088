"""ImageNet stem kernels (csrc/kernels/stem.hip) against fp32 torch: the direct 7x7 / stride-2 / pad-3 conv
with BN statistics (odd sizes, partial last tile, zero-padded channels) and the fused BN-apply + ReLU +
3x3/s2 max-pool (bitwise equal to bn_apply followed by maxpool_fwd, same argmax)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


@pytest.fixture(scope="module")
def K():
    from pytorch_distributed_nn_amd.ops import kernels, _backend
    assert _backend.available()
    return kernels


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


@pytest.mark.parametrize("shape", [(2, 224, 224), (3, 37, 53), (1, 8, 8), (5, 64, 64), (1, 1, 1)])
def test_stem_conv_matches_fp32(K, shape):
    N, H, W = shape
    x = torch.zeros(N, H, W, 8, device="cuda")
    x[..., :3] = torch.randn(N, H, W, 3, device="cuda")
    x = x.to(BF)
    w = torch.zeros(64, 7, 7, 8, device="cuda")
    w[..., :3] = torch.randn(64, 7, 7, 3, device="cuda") * 0.1
    w = w.to(BF)
    assert K.stem_ok(x.shape, w.shape, 2, 3)
    y, slab = K.stem_conv(x, w)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), None, 2, 3).permute(0, 2, 3, 1)
    assert y.shape == ref.shape
    assert rel(y, ref) < 1e-2
    yf = y.float().reshape(-1, 64)
    s = slab.view(-1, 2, 64).sum(0)
    assert torch.allclose(s[0], yf.sum(0), rtol=1e-3, atol=1e-2 * yf.abs().max().item())
    assert torch.allclose(s[1], (yf * yf).sum(0), rtol=1e-3, atol=1e-1)
    # the generic implicit-GEMM path agrees
    y2, _ = K.conv_fwd(x, w, 2, 3, want_stats=True)
    assert rel(y, y2) < 1e-2


@pytest.mark.parametrize("shape", [(2, 112, 112, 64), (3, 15, 9, 64), (1, 2, 2, 16), (2, 7, 8, 8)])
def test_bn_relu_maxpool_bitwise(K, shape):
    N, H, W, C = shape
    t = torch.randn(N, H, W, C, device="cuda").to(BF)
    sc, sh = torch.randn(C, device="cuda"), torch.randn(C, device="cuda") * 0.5
    y, idx = K.bn_relu_maxpool(t, sc, sh)
    a = K.bn_apply(t.view(-1, C), sc, sh, relu=True)
    a = (a[0] if isinstance(a, tuple) else a).view(t.shape)
    y_ref, idx_ref = K.maxpool_fwd(a, 3, 2, 1)
    assert torch.equal(y, y_ref)
    assert torch.equal(idx, idx_ref)


@pytest.mark.parametrize("shape", [(2, 224, 224), (3, 38, 52), (1, 8, 8), (4, 64, 64), (1, 9, 10)])
def test_stem_conv_nchw_matches_fp32(K, shape):
    """The stem conv straight from the NCHW bf16 batch (k = channel*8 + column, border columns word-shifted)."""
    N, H, W = shape
    x = torch.randn(N, 3, H, W, device="cuda").to(BF)
    w = torch.randn(64, 3, 7, 7, device="cuda") * 0.1
    assert K.stem_nchw_ok(x)
    y, slab = K.stem_conv_nchw(x, K.stem_weight_nchw(w))
    ref = F.conv2d(x.float(), w.to(BF).float(), None, 2, 3).permute(0, 2, 3, 1)
    assert y.shape == ref.shape
    assert rel(y, ref) < 1e-2
    yf = y.float().reshape(-1, 64)
    s = slab.view(-1, 2, 64).sum(0)
    assert torch.allclose(s[0], yf.sum(0), rtol=1e-3, atol=1e-2 * yf.abs().max().item())
    assert torch.allclose(s[1], (yf * yf).sum(0), rtol=1e-3, atol=1e-1)


@pytest.mark.parametrize("shape", [(4, 64, 64), (2, 224, 224)])
def test_stem_fn_modes_agree(K, shape):
    """StemFn (conv + BN + ReLU + max-pool, and its backward) with the NCHW kernel (K.set_stem_mode 2), the NHWC
    direct kernel (1) and the generic path (0), same input and upstream gradient: outputs within bf16 rounding
    (different summation orders flip a few last bits), parameter gradients aligned."""
    from pytorch_distributed_nn_amd.ops import functional as OF
    from pytorch_distributed_nn_amd.ops.fused_resnet import StemFn, stem_shadow
    N, H, W = shape
    torch.manual_seed(0)
    x = torch.randn(N, 3, H, W, device="cuda").to(BF)
    w = (torch.randn(64, 3, 7, 7, device="cuda") * 0.1).requires_grad_()
    gamma = (torch.rand(64, device="cuda") + 0.5).requires_grad_()
    beta = (torch.randn(64, device="cuda") * 0.1).requires_grad_()
    gy = None
    res = {}
    for mode in (2, 1, 0):
        old = K.set_stem_mode(mode)
        try:
            bufs = [torch.zeros(64, device="cuda"), torch.ones(64, device="cuda")]
            conf = (2, 3, True, True, 0.1, 1e-5)
            if mode == 2:
                y = StemFn.apply(x.contiguous(), conf, bufs, [K.stem_weight_nchw(w)], w, gamma, beta)
            else:
                xin = OF.nchw_to_nhwc_input(x)
                y = StemFn.apply(xin, conf, bufs, [stem_shadow(w, 8)], w, gamma, beta)
            if gy is None:
                gy = torch.randn_like(y.float()).to(BF)
            dw, dg, db = torch.autograd.grad(y, (w, gamma, beta), gy)
            torch.cuda.synchronize()
            res[mode] = (y.float(), dw, dg, db, bufs)
        finally:
            K.set_stem_mode(old)
    y0, dw0, dg0, db0, b0 = res[0]
    assert torch.equal(res[1][0], y0)               # NHWC direct kernel: same summation order as the engine
    for mode in (2, 1):
        y, dw, dg, db, b = res[mode]
        assert (y - y0).abs().max() <= 2 ** -6 * y0.abs().max()       # a few last-bit flips at most
        assert (y != y0).float().mean() < 1e-3
        for a, r in ((dw, dw0), (dg, dg0), (db, db0)):
            assert torch.nn.functional.cosine_similarity(a.flatten(), r.flatten(), dim=0) > 0.999
        torch.testing.assert_close(b[0], b0[0], rtol=1e-3, atol=1e-4)     # running statistics


def test_stem_eval_mode_without_statistics(K):
    """want_stats=False (eval-mode BatchNorm) takes the plain epilogue: same output, no slab."""
    x = torch.randn(2, 3, 40, 48, device="cuda").to(BF)
    w = torch.randn(64, 3, 7, 7, device="cuda") * 0.1
    y1, s1 = K.stem_conv_nchw(x, K.stem_weight_nchw(w))
    y0, s0 = K.stem_conv_nchw(x, K.stem_weight_nchw(w), want_stats=False)
    assert s0 is None and torch.equal(y0, y1)
    xin = K.nchw_to_nhwc(x, 8)
    kpad = torch.nn.functional.pad(w.to(BF).permute(0, 2, 3, 1), (0, 5)).contiguous()
    z1, _ = K.stem_conv(xin, kpad)
    z0, t0 = K.stem_conv(xin, kpad, want_stats=False)
    assert t0 is None and torch.equal(z0, z1)


def test_resnet50_eval_forward_uses_direct_stem(K):
    from pytorch_distributed_nn_amd.models import build_model
    torch.manual_seed(0)
    m = build_model("resnet50").cuda().eval()
    x = torch.randn(2, 3, 64, 64, device="cuda").to(BF)
    with torch.no_grad():
        out = m(x)
    torch.cuda.synchronize()
    assert torch.isfinite(out.float()).all()


@pytest.mark.parametrize("shape", [(4, 64, 64), (2, 224, 224), (3, 30, 18), (1, 9, 8)])
def test_stem_wgrad_nchw_matches_fp32(K, shape):
    """Weight gradient of the NCHW stem (stem_wgrad.hip: NCHW batch read directly, transpose-read reduction over
    the pixels) against fp32 torch, including partial last tiles and border columns."""
    N, H, W = shape
    x = torch.randn(N, 3, H, W, device="cuda").to(BF)
    w = torch.zeros(64, 3, 7, 7, device="cuda", requires_grad=True)
    y = F.conv2d(x.float(), w, None, 2, 3)
    dt = torch.randn(*y.permute(0, 2, 3, 1).shape, device="cuda").to(BF)
    y.backward(dt.float().permute(0, 3, 1, 2))
    dw = K.stem_wgrad_nchw(x, dt.contiguous())
    assert dw.shape == (64, 3, 7, 7)
    assert rel(dw, w.grad) < 5e-3, rel(dw, w.grad)


@pytest.mark.parametrize("shape", [(4, 64, 64), (3, 30, 18)])
def test_stem_wgrad_nchw_fused_bn_apply(K, shape):
    """The BN-backward apply (mask mode 2) inside the NCHW stem weight-gradient staging == apply pass + kernel."""
    N, H, W = shape
    x = torch.randn(N, 3, H, W, device="cuda").to(BF)
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    ga = torch.randn(N, Ho, Wo, 64, device="cuda").to(BF)
    t = torch.randn(N, Ho, Wo, 64, device="cuda").to(BF)
    mean, inv = torch.randn(64, device="cuda") * 0.1, torch.rand(64, device="cuda") + 0.5
    gamma = torch.rand(64, device="cuda") + 0.5
    dg, db = torch.randn(64, device="cuda") * 50, torch.randn(64, device="cuda") * 50
    s, h = torch.rand(64, device="cuda") + 0.5, torch.randn(64, device="cuda") * 0.3
    dt = K.bn_bwd_apply(ga.view(-1, 64), t.view(-1, 64), mean, inv, gamma, dg, db, mode=2, msrc=t.view(-1, 64),
                        mscale=s, mshift=h)[0].view_as(ga)
    ref = K.stem_wgrad_nchw(x, dt)
    out = K.stem_wgrad_nchw(x, ga, pre=(t, mean, inv, gamma, dg, db, s, h))
    assert rel(out, ref) < 1e-5, rel(out, ref)


@pytest.mark.parametrize("shape", [(2, 112, 112, 64), (3, 16, 10, 64), (1, 2, 2, 16), (2, 8, 6, 8)])
def test_maxpool_bwd_bnred_matches_two_passes(K, shape):
    """The stem's fused max-pool gather + mode-2 BN-backward reduce (pool.hip maxpool_bwd_bnred_kernel): the
    pooled gradient is bitwise maxpool_bwd's, the summed slab matches bn_bwd_reduce(mode=2) on it."""
    N, H, W, C = shape
    t = torch.randn(N, H, W, C, device="cuda").to(BF)
    sc, sh = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.5
    mean, inv = torch.randn(C, device="cuda") * 0.1, torch.rand(C, device="cuda") + 0.5
    y, idx = K.bn_relu_maxpool(t, sc, sh)
    gy = torch.randn_like(y.float()).to(BF)
    ga_ref = K.maxpool_bwd(gy, idx, t.shape, 3, 2, 1)
    slab_ref, _, rows_ref = K.bn_bwd_reduce(ga_ref.view(-1, C), t.view(-1, C), mean, inv, mode=2,
                                            msrc=t.view(-1, C), mscale=sc, mshift=sh)
    out = K.maxpool_bwd_bnred(gy, idx, t, mean, inv, sc, sh)
    assert out is not None
    ga, slab, rows = out
    assert torch.equal(ga, ga_ref)
    a = slab.view(rows, 2, C).double().sum(0)
    b = slab_ref.view(rows_ref, 2, C).double().sum(0)
    torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-3)


def test_maxpool_bwd_bnred_declines_odd_sizes(K):
    t = torch.randn(1, 9, 8, 64, device="cuda").to(BF)
    y, idx = K.bn_relu_maxpool(t, torch.ones(64, device="cuda"), torch.zeros(64, device="cuda"))
    z = torch.zeros(64, device="cuda")
    assert K.maxpool_bwd_bnred(y, idx, t, z, z, z, z) is None


def test_stem_wgrad_nchw_accumulates_into_channels_last_grad(K):
    """acc=: the reduce adds the weight gradient straight into a [64,3,7,7] channels-last fp32 gradient (the
    flat arena's view of the stem weight) instead of returning it."""
    x = torch.randn(3, 3, 30, 18, device="cuda").to(BF)
    dt = torch.randn(3, 15, 9, 64, device="cuda").to(BF)
    ref = K.stem_wgrad_nchw(x, dt)
    base = torch.randn(64, 3, 7, 7, device="cuda").contiguous(memory_format=torch.channels_last)
    acc = base.clone()
    assert acc.stride() == (147, 1, 21, 3)
    assert K.stem_wgrad_nchw(x, dt, acc=acc) is None
    torch.testing.assert_close(acc, base + ref, rtol=1e-5, atol=1e-5)
