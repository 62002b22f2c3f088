"""Numerics of every HIP kernel against a plain PyTorch fp32 reference of the same op (SURVEY.md §7.4
``tests/kernels``).  Inputs are rounded to bf16 first so the reference sees exactly what the kernel sees;
tolerances are relative to the reference's max magnitude (bf16 output rounding is ~4e-3)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

BF = torch.bfloat16


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


@pytest.fixture(scope="module")
def K():
    from pytorch_distributed_nn_amd.ops import kernels, _backend
    assert _backend.available(), "HIP kernel library must load on a GPU box"
    return kernels


@pytest.fixture(autouse=True, params=[(1, 1, 1), (0, 1, 0), (0, 0, 0), (2, 1, 0), (1, 1, 2)],
                ids=["auto", "reg128", "reg128-direct-store", "glds", "pp"])
def engine(request, K):
    """Every GEMM/conv test runs with automatic engine choice, the register-staged 128-tile kernel only
    (LDS-staged and direct epilogue stores), the glds 256-row engine forced wherever it applies, and the
    ping-pong engine forced wherever it applies (plain GEMMs, 1x1 stride-1 convs with their fusions)."""
    glds, staged, pp = request.param
    old = K.set_glds_mode(glds)
    old_s = K.set_staged_store(staged)
    old_p = K.set_pp_mode(pp)
    yield request.param
    K.set_glds_mode(old)
    K.set_staged_store(old_s)
    K.set_pp_mode(old_p)


def rnd(*s, scale=1.0):
    return (torch.randn(*s, device="cuda") * scale).to(BF)


@pytest.mark.parametrize("M,N,Kd", [(256, 256, 256), (200, 136, 72), (1000, 1000, 2048), (64, 8, 8), (4096, 768, 3072)])
def test_gemm_nt(K, M, N, Kd):
    x, w = rnd(M, Kd), rnd(N, Kd)
    b = torch.randn(N, device="cuda")
    y = K.gemm_nt(x, w, bias=b)
    ref = x.float() @ w.float().t() + b
    assert rel(y, ref) < 1e-2
    y32 = K.gemm_nt(x, w, out_f32=True, relu=True)
    assert rel(y32, F.relu(x.float() @ w.float().t())) < 2e-3


@pytest.mark.parametrize("M,N,Kd", [(256, 256, 256), (200, 136, 72), (512, 2048, 1000)])
def test_gemm_nn(K, M, N, Kd):
    x, w = rnd(M, Kd), rnd(Kd, N)
    y = K.gemm_nn(x, w)
    assert rel(y, x.float() @ w.float()) < 1e-2


@pytest.mark.parametrize("M,N,Kd", [(256, 256, 256), (136, 200, 72), (1000, 2048, 256), (768, 3072, 8192)])
def test_gemm_tn_acc(K, M, N, Kd):
    x, y = rnd(Kd, M), rnd(Kd, N)
    out = torch.zeros(M, N, device="cuda")
    K.gemm_tn_acc(x, y, out)
    assert rel(out, x.float().t() @ y.float()) < 2e-3


CONV_SHAPES = [
    # N, H, W, C, Ko, R, stride, pad
    (2, 8, 8, 64, 64, 1, 1, 0),
    (2, 9, 9, 64, 128, 3, 1, 1),
    (2, 14, 14, 128, 128, 3, 2, 1),
    (2, 14, 14, 256, 512, 1, 2, 0),
    (2, 32, 32, 8, 64, 7, 2, 3),
    (3, 7, 7, 512, 2048, 1, 1, 0),
    (2, 56, 56, 64, 256, 1, 1, 0),
    (2, 15, 15, 64, 64, 3, 2, 1),
    (2, 15, 15, 64, 128, 1, 2, 0),
    (3, 10, 10, 64, 128, 3, 1, 1),       # M = 300: ragged 256-row tiles, partial stats groups
    (2, 12, 12, 128, 64, 3, 2, 1),
    (32, 56, 56, 64, 64, 3, 1, 1),       # 392 row tiles: the persistent glds grid loops over tiles
]


def conv_ref(x, w, st, pad):
    # x NHWC, w [K][R][S][C]
    return F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), None, st, pad).permute(0, 2, 3, 1)


@pytest.mark.parametrize("shape", CONV_SHAPES)
@pytest.mark.parametrize("pro", [False, True])
def test_conv_fwd(K, shape, pro):
    N, H, W, C, Ko, R, st, pad = shape
    x, w = rnd(N, H, W, C), rnd(Ko, R, R, C, scale=0.1)
    prolog = None
    xin = x
    if pro:
        sc, sh = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.2
        prolog = (sc, sh)
        xin = F.relu(x.float() * sc + sh).to(BF)
    y, stats = K.conv_fwd(x, w, st, pad, pro=prolog, want_stats=True)
    ref = conv_ref(xin, w, st, pad)
    assert y.shape == ref.shape
    assert rel(y, ref) < 1.5e-2
    # fused BN partial statistics of the bf16 output
    yf = y.float().reshape(-1, Ko)
    s = stats.view(-1, 2, Ko).sum(0)
    assert torch.allclose(s[0], yf.sum(0), rtol=1e-3, atol=1e-2 * yf.abs().max().item())
    assert torch.allclose(s[1], (yf * yf).sum(0), rtol=1e-3, atol=1e-1)


@pytest.mark.parametrize("shape", CONV_SHAPES)
def test_conv_dgrad(K, shape):
    N, H, W, C, Ko, R, st, pad = shape
    x = torch.randn(N, C, H, W, device="cuda", requires_grad=True)
    w = rnd(Ko, R, R, C, scale=0.1)
    y = F.conv2d(x, w.float().permute(0, 3, 1, 2), None, st, pad)
    dy = rnd(*y.permute(0, 2, 3, 1).shape)
    y.backward(dy.float().permute(0, 3, 1, 2))
    dx = K.conv_dgrad(dy, w, (N, H, W, C), st, pad)
    assert rel(dx, x.grad.permute(0, 2, 3, 1)) < 1.5e-2
    # in-place accumulation (shortcut branch of a residual block): out aliases res; a strided conv only
    # touches the pixels its taps reach, every other pixel must keep res
    base = rnd(N, H, W, C)
    acc = base.clone()
    K.conv_dgrad(dy, w, (N, H, W, C), st, pad, res=acc, out=acc)
    assert rel(acc, base.float() + x.grad.permute(0, 2, 3, 1)) < 1.5e-2


@pytest.mark.parametrize("shape", CONV_SHAPES)
@pytest.mark.parametrize("pro", [False, True])
def test_conv_wgrad(K, shape, pro):
    N, H, W, C, Ko, R, st, pad = shape
    x = rnd(N, H, W, C)
    xin = x
    prolog = None
    if pro:
        sc, sh = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.2
        prolog = (sc, sh)
        xin = F.relu(x.float() * sc + sh).to(BF)
    w = torch.zeros(Ko, C, R, R, device="cuda", requires_grad=True)
    y = F.conv2d(xin.float().permute(0, 3, 1, 2), w, None, st, pad)
    dy = rnd(*y.permute(0, 2, 3, 1).shape)
    y.backward(dy.float().permute(0, 3, 1, 2))
    dw = K.conv_wgrad(x, dy, R, R, st, pad, pro=prolog)
    assert rel(dw, w.grad.permute(0, 2, 3, 1)) < 5e-3


@pytest.mark.parametrize("C", [8, 64, 200, 256, 1024, 2048])
def test_bn_bins_finalize(K, C):
    """Finalize of the 64 statistics bins (one block per 64-channel column, fp64 sums) against fp64 torch sums;
    several calls in a row, and the bins come back zeroed for the next producer."""
    rows = K.STAT_BINS
    L = float(rows * 64)
    for it in range(4):
        slab = torch.rand(rows, 2, C, device="cuda") * 64
        slab[:, 1] += slab[:, 0] ** 2 / 64 + 1.0            # sum of squares consistent with a positive var
        slab = slab.reshape(rows * 2, C)
        sd = slab.view(rows, 2, C).double().sum(0)
        gamma, beta = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda")
        rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        mean, inv, sc, sh = K.bn_finalize(slab, rows, L, 1e-5, 0.1, gamma, beta, rm, rv)
        m_ref = sd[0] / L
        v_ref = (sd[1] / L - m_ref ** 2).clamp_min(0)
        assert torch.allclose(mean.double(), m_ref, rtol=1e-5, atol=1e-6)
        assert torch.allclose(inv.double(), torch.rsqrt(v_ref + 1e-5), rtol=1e-4)
        assert torch.allclose(sc.double(), gamma.double() * torch.rsqrt(v_ref + 1e-5), rtol=1e-4)
        assert torch.allclose(rm.double(), 0.1 * m_ref, rtol=1e-5, atol=1e-6)
        assert not slab.any()                                  # zeroed for the next producer
        slab.copy_(torch.rand(rows * 2, C, device="cuda"))
        sd = slab.view(rows, 2, C).double().sum(0)
        dg, db = torch.full((C,), 1.0, device="cuda"), torch.full((C,), 2.0, device="cuda")
        acc = (torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda"))
        K.bn_bwd_finalize(slab, rows, dg, db, accumulate=True, acc=acc)
        assert torch.allclose(db.double(), sd[0] + 2.0, rtol=1e-5)
        assert torch.allclose(dg.double(), sd[1] + 1.0, rtol=1e-5)
        assert torch.allclose(acc[0].double(), sd[1], rtol=1e-5) and torch.allclose(acc[1].double(), sd[0], rtol=1e-5)
        assert not slab.any()


def test_bn_bins_pool_two_streams_many_calls(K):
    """200 reduce -> finalize pairs alternating between two streams with no synchronisation between them: the
    zeroed-bins free list is per stream, so a slab is reused only behind the finalize that zeroed it."""
    streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
    streams[1].wait_stream(streams[0])
    outs = []
    g = torch.Generator(device="cuda").manual_seed(0)
    for i in range(200):
        L, C = (4096, 256) if i % 3 else (8192, 64)
        st = streams[i % 2]
        with torch.cuda.stream(st):
            x = torch.randn(L, C, device="cuda", generator=g).to(torch.bfloat16)
            slab, rows = K.bn_stats(x)
            dg, db = K.bn_bwd_finalize(slab, rows)
        outs.append((x, dg, db))
    torch.cuda.synchronize()
    for x, dg, db in outs:
        xf = x.double()
        assert torch.allclose(db.double(), xf.sum(0), rtol=1e-4, atol=1e-2)
        assert torch.allclose(dg.double(), (xf * xf).sum(0), rtol=1e-4)


def test_bn_train_fwd_bwd(K):
    L, C = 4096, 256
    x = rnd(L, C, scale=2.0) + 0.5
    gamma, beta = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda")
    rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    slab, rows = K.bn_stats(x)
    mean, inv, sc, sh = K.bn_finalize(slab, rows, L, 1e-5, 0.1, gamma, beta, rm, rv)
    xf = x.float()
    assert torch.allclose(mean, xf.mean(0), atol=1e-3)
    assert torch.allclose(inv, torch.rsqrt(xf.var(0, unbiased=False) + 1e-5), rtol=1e-3)
    assert torch.allclose(rv, 0.9 + 0.1 * xf.var(0, unbiased=True), rtol=1e-3)
    y = K.bn_apply(x, sc, sh, relu=True)
    xr = xf.clone().requires_grad_(True)
    g_, b_ = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    ref = F.relu(F.batch_norm(xr, None, None, g_, b_, True, 0.1, 1e-5))
    assert rel(y, ref) < 1e-2
    gy = rnd(L, C)
    ref.backward(gy.float())
    slab, _, rows = K.bn_bwd_reduce(gy, x, mean, inv, mode=1, msrc=y)
    dg, db = K.bn_bwd_finalize(slab, rows)
    dx, _, _ = K.bn_bwd_apply(gy, x, mean, inv, gamma, dg, db, mode=1, msrc=y)
    assert rel(dg, g_.grad) < 2e-2 and rel(db, b_.grad) < 2e-2
    assert rel(dx, xr.grad) < 3e-2
    # mask mode 3: the ReLU mask as sign bits written by bn_apply, bit-exact with mode 1 on y
    y3, bits = K.bn_apply(x, sc, sh, relu=True, want_mask=True)
    assert torch.equal(y3, y) and bits.shape == (L, C // 8) and bits.dtype == torch.uint8
    ref_bits = ((y.view(L, C // 8, 8) > 0).to(torch.int32) << torch.arange(8, device="cuda")).sum(-1)
    assert torch.equal(bits.to(torch.int32), ref_bits)
    slab3, _, rows3 = K.bn_bwd_reduce(gy, x, mean, inv, mode=3, msrc=bits)
    dg3, db3 = K.bn_bwd_finalize(slab3, rows3)
    # the statistics are fp32 atomic sums (summation order varies): equal to mode 1 up to rounding
    assert torch.allclose(dg3, dg, rtol=1e-5, atol=1e-4) and torch.allclose(db3, db, rtol=1e-5, atol=1e-4)
    dx3, _, _ = K.bn_bwd_apply(gy, x, mean, inv, gamma, dg, db, mode=3, msrc=bits)
    assert torch.equal(dx3, dx)


@pytest.mark.parametrize("k,st,pad", [(3, 2, 1), (2, 2, 0), (3, 1, 1), (5, 2, 2)])
def test_maxpool(K, k, st, pad):
    x = torch.randn(2, 17, 17, 64, device="cuda").to(BF).requires_grad_(False)
    y, idx = K.maxpool_fwd(x, k, st, pad)
    xr = x.float().permute(0, 3, 1, 2).clone().requires_grad_(True)
    ref = F.max_pool2d(xr, k, st, pad)
    assert rel(y, ref.permute(0, 2, 3, 1)) < 1e-6
    g = rnd(*y.shape)
    ref.backward(g.float().permute(0, 3, 1, 2))
    dx = K.maxpool_bwd(g, idx, x.shape, k, st, pad)
    assert rel(dx, xr.grad.permute(0, 2, 3, 1)) < 1e-2


def test_avgpool(K):
    x = rnd(4, 7, 7, 2048)
    y = K.avgpool_fwd(x)
    assert rel(y, x.float().mean((1, 2))) < 1e-2
    g = rnd(4, 2048)
    dx = K.avgpool_bwd(g, x.shape)
    assert rel(dx, (g.float() / 49)[:, None, None, :].expand(4, 7, 7, 2048)) < 1e-2


@pytest.mark.parametrize("V", [10, 1000, 50257, 50304, 8])
def test_xent(K, V):
    R = 64
    lg = rnd(R, V, scale=3.0)
    y = torch.randint(0, V, (R,), device="cuda")
    y[3] = -100
    loss, lse, acc = K.xent_fwd(lg, y)
    lr = lg.float().clone().requires_grad_(True)
    ref = F.cross_entropy(lr, y, reduction="sum")
    assert abs(acc[0].item() - ref.item()) / abs(ref.item()) < 1e-4
    ref.backward()
    gs = torch.ones(1, device="cuda")
    d = K.xent_bwd(lg, y, lse, gs, 1.0)
    assert rel(d, lr.grad) < 1e-2
    # mean reduction: the scale g / max(count, 1) formed in the kernel from the forward's device-side count
    assert acc[1].item() == R - 1
    dm = K.xent_bwd(lg, y, lse, gs, 1.0, count=acc[1:2])
    assert rel(dm, lr.grad / (R - 1)) < 1e-2
    # training forward with the unscaled gradient written in place (bf16, V % 8 == 0 only)
    if V % 8 == 0:
        lg2 = lg.clone()
        loss2, lse2, acc2, d2 = K.xent_fwd_grad(lg2, y)
        assert d2.data_ptr() == lg2.data_ptr()
        assert rel(lse2, lse) < 1e-5 and rel(loss2, loss) < 1e-4
        assert acc2[1].item() == acc[1].item() and rel(acc2[:1], acc[:1]) < 1e-5
        assert rel(d2, lr.grad) < 1e-2 and d2[3].abs().max().item() == 0.0


def test_sgd_adam(K):
    n = 10007
    p, g = torch.randn(n, device="cuda"), torch.randn(n, device="cuda")
    buf = torch.zeros(n, device="cuda")
    sh = torch.empty(n, device="cuda", dtype=BF)
    pr = p.clone().requires_grad_(True)
    opt = torch.optim.SGD([pr], lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=True)
    for first in (True, False):
        pr.grad = g.clone()
        opt.step()
        K.sgd_step(p, g, buf, sh, 0.1, 0.9, 0.0, 1e-4, True, first=first)
    assert torch.allclose(p, pr.detach(), atol=1e-6)
    assert rel(sh, p) < 5e-3
    p2 = torch.randn(n, device="cuda")
    m, v = torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
    pr2 = p2.clone().requires_grad_(True)
    opt2 = torch.optim.AdamW([pr2], lr=1e-3, weight_decay=0.01)
    for t in (1, 2, 3):
        pr2.grad = g.clone()
        opt2.step()
        K.adam_step(p2, g, m, v, None, 1e-3, 0.9, 0.999, 1e-8, 0.01, True, 1 - 0.9 ** t, 1 - 0.999 ** t)
    assert torch.allclose(p2, pr2.detach(), atol=1e-6)


@pytest.mark.parametrize("offset", [0, 1])          # 16-B aligned float4 body + tail / scalar-only path
def test_adam_vec_and_device_hyper(K, offset):
    """Adam over an (un)aligned slice with bf16 shadow, hyper-parameters read from device memory
    (graph-replay mode) vs torch.optim.Adam; SGD lr from device memory vs by value."""
    n = 4099
    base = torch.randn(n + offset, device="cuda")
    p = base[offset:]
    g = torch.randn(n, device="cuda")
    m, v = torch.zeros(n + offset, device="cuda")[offset:], torch.zeros(n + offset, device="cuda")[offset:]
    sh = torch.empty(n + offset, device="cuda", dtype=BF)[offset:]
    pr = p.clone().requires_grad_(True)
    opt = torch.optim.Adam([pr], lr=2e-3, weight_decay=0.01)
    hyper = torch.zeros(3, device="cuda")
    for t in (1, 2, 3):
        pr.grad = g.clone()
        opt.step()
        hyper.copy_(torch.tensor([2e-3, 1 - 0.9 ** t, 1 - 0.999 ** t]))
        # by-value lr/bc deliberately wrong: the device values must win
        K.adam_step(p, g, m, v, sh, 9.0, 0.9, 0.999, 1e-8, 0.01, False, 0.5, 0.5, hyper=hyper)
    assert torch.allclose(p, pr.detach(), atol=1e-6)
    assert rel(sh, p) < 5e-3
    q1, q2 = torch.randn(n, device="cuda"), None
    q2 = q1.clone()
    b1, b2 = torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
    lr_dev = torch.tensor([0.05], device="cuda")
    for first in (True, False):
        K.sgd_step(q1, g, b1, None, 0.05, 0.9, 0.0, 0.0, False, first=first)
        K.sgd_step(q2, g, b2, None, 7.0, 0.9, 0.0, 0.0, False, first=first, hyper=lr_dev)
    assert torch.equal(q1, q2)


@pytest.mark.parametrize("op", ["relu", "sigmoid", "gelu"])
def test_act(K, op):
    x = rnd(4096)
    y = K.act_fwd(x, op)
    xr = x.float().clone().requires_grad_(True)
    f = {"relu": F.relu, "sigmoid": torch.sigmoid, "gelu": lambda t: F.gelu(t, approximate="tanh")}[op]
    r = f(xr)
    assert rel(y, r) < 1e-2
    g = rnd(4096)
    r.backward(g.float())
    assert rel(K.act_bwd(g, x, op), xr.grad) < 2e-2


@pytest.mark.parametrize("shape", [(2, 14, 14, 128, 128, 3, 2, 1), (2, 9, 9, 64, 128, 3, 1, 1), (2, 8, 8, 256, 64, 1, 1, 0)])
def test_conv_dgrad_fused_bn_backward_and_residual(K, shape):
    """dgrad epilogue fusions: residual add, and BN-backward ReLU masking + reduction (sum gm, sum gm*xhat)."""
    N, H, W, C, Ko, R, st, pad = shape
    w = rnd(Ko, R, R, C, scale=0.1)
    Ho, Wo = K.conv_out_hw(H, W, R, R, st, pad)
    dy = rnd(N, Ho, Wo, Ko)
    x = torch.zeros(N, C, H, W, device="cuda", requires_grad=True)
    y = F.conv2d(x, w.float().permute(0, 3, 1, 2), None, st, pad)
    y.backward(dy.float().permute(0, 3, 1, 2))
    dx_ref = x.grad.permute(0, 2, 3, 1)
    res = rnd(N, H, W, C)
    dx = K.conv_dgrad(dy, w, (N, H, W, C), st, pad, res=res)
    assert rel(dx, dx_ref + res.float()) < 1.5e-2
    t = rnd(N, H, W, C) + 0.3
    mean, inv = torch.randn(C, device="cuda") * 0.1, torch.rand(C, device="cuda") + 0.5
    sc, sh = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.3
    gm, slab = K.conv_dgrad(dy, w, (N, H, W, C), st, pad, bn=(t, mean, inv, sc, sh))
    mask = (t.float() * sc + sh) > 0
    gm_ref = dx_ref.to(BF).float() * mask
    assert rel(gm, gm_ref) < 1.5e-2
    sums = slab.view(-1, 2, C).sum(0)
    xh = (t.float() - mean) * inv
    # norm-relative: the reference sums bf16-rounded gm, the kernel its fp32 values, so a channel whose sum
    # lands near zero can miss any per-element atol (unseeded inputs; r4_71)
    assert rel(sums[0], gm_ref.reshape(-1, C).sum(0)) < 1e-2
    assert rel(sums[1], (gm_ref * xh).reshape(-1, C).sum(0)) < 1e-2


@pytest.mark.parametrize("shape", [(16, 28, 28, 128, 512, False), (16, 28, 28, 512, 128, True),
                                   (4, 14, 14, 1024, 256, True), (3, 10, 10, 256, 128, True),
                                   (8, 14, 14, 256, 1024, False), (5, 7, 7, 512, 2048, False)])
def test_conv1x1_fused_resnet_shapes(K, shape):
    """1x1 stride-1 convs at bottleneck shapes (the ping-pong engine in auto mode): forward with the
    BN-affine+ReLU prologue and BN statistics; data gradient with residual, and with the BN-backward
    masking + reduction epilogue."""
    N, H, W, C, Ko, pro = shape
    x, w = rnd(N, H, W, C), rnd(Ko, 1, 1, C, scale=0.1)
    prolog, xin = None, x
    if pro:
        sc, sh = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.2
        prolog, xin = (sc, sh), F.relu(x.float() * sc + sh).to(BF)
    y, stats = K.conv_fwd(x, w, 1, 0, pro=prolog, want_stats=True)
    ref = conv_ref(xin, w, 1, 0)
    assert rel(y, ref) < 1.5e-2
    yf = y.float().reshape(-1, Ko)
    s = stats.view(-1, 2, Ko).sum(0)
    assert torch.allclose(s[0], yf.sum(0), rtol=1e-3, atol=1e-2 * yf.abs().max().item())
    assert torch.allclose(s[1], (yf * yf).sum(0), rtol=1e-3, atol=1e-1)
    # data gradient: dy [N,H,W,Ko] -> dx [N,H,W,C]
    dy = rnd(N, H, W, Ko)
    dx_ref = (dy.float().reshape(-1, Ko) @ w.float().reshape(Ko, C)).view(N, H, W, C)
    res = rnd(N, H, W, C)
    assert rel(K.conv_dgrad(dy, w, (N, H, W, C), 1, 0, res=res), dx_ref + res.float()) < 1.5e-2
    t = rnd(N, H, W, C) + 0.3
    mean, inv = torch.randn(C, device="cuda") * 0.1, torch.rand(C, device="cuda") + 0.5
    bsc, bsh = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.3
    gm, slab = K.conv_dgrad(dy, w, (N, H, W, C), 1, 0, bn=(t, mean, inv, bsc, bsh))
    z = t.float() * bsc + bsh
    gm_ref = dx_ref.to(BF).float() * (z > 0)
    sure = z.abs() > 1e-4          # the kernel evaluates the mask with one fma: skip sign ties
    assert rel(gm.float() * sure, gm_ref * sure) < 1.5e-2
    sums = slab.view(-1, 2, C).sum(0)
    xh = (t.float() - mean) * inv
    tol = 1e-2 * gm_ref.abs().sum(dim=(0, 1, 2)).max().item() / 10
    assert torch.allclose(sums[0], gm_ref.reshape(-1, C).sum(0), atol=max(tol, 5e-2), rtol=1e-2)
    assert torch.allclose(sums[1], (gm_ref * xh).reshape(-1, C).sum(0), atol=max(tol, 5e-2), rtol=1e-2)


@pytest.mark.parametrize("R,C", [(100, 10), (8192, 768), (8192, 3072), (3000, 2304), (513, 40), (260, 1032), (100000, 64),
                                 (8191, 2312)])
def test_colsum(K, R, C):
    x = rnd(R, C)
    out = K.colsum(x)
    ref = x.float().sum(0)
    assert rel(out, ref) < 1e-4
    K.colsum(x, out=out, accumulate=True)                       # tall shapes: one-launch atomic form
    assert rel(out, 2 * ref) < 1e-4
    K.colsum(x, out=out, accumulate=True, deterministic=True)   # two-level form
    assert rel(out, 3 * ref) < 1e-4


@pytest.mark.parametrize("Kd,M,N,splits", [(8192, 3072, 768, None), (8192, 768, 3072, 3), (8192, 768, 768, 14),
                                           (1024, 768, 768, 5), (96, 520, 264, 2), (8192, 2304, 768, 1)])
def test_pp_wgrad_uneven_splits(K, Kd, M, N, splits):
    """out += x^T y on the ping-pong engine; split counts that do not divide the K slices give the first
    splits one slice more (every slice summed exactly once)."""
    x, y = rnd(Kd, M), rnd(Kd, N)
    out = torch.randn(M, N, device="cuda")
    ref = out + x.float().t() @ y.float()
    K.pp_wgrad(x, y, out, splits=splits)
    assert rel(out, ref) < 2e-5
    # the fused row sums (a linear layer's bias gradient beside its weight gradient), accumulated
    rs = torch.randn(M, device="cuda")
    rs_ref = rs + x.float().sum(0)
    out2 = torch.zeros(M, N, device="cuda")
    K.pp_wgrad(x, y, out2, splits=splits, rowsum=rs)
    assert rel(out2, x.float().t() @ y.float()) < 2e-5
    assert rel(rs, rs_ref) < 2e-5
    # fp32 epilogues through buffer stores with the drain deferred (pp_epi_slack 2): the same bits
    outs = []
    for sl in (1, 2):
        old = K.tune_set("pp_epi_slack", sl)
        try:
            o = out.clone()
            K.pp_wgrad(x, y, o, splits=splits)
            outs.append(o)
        finally:
            K.tune_set("pp_epi_slack", old)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("bn,form", [(96, "sk64"), (96, "sk32"), (128, "sk64"), (128, "sk32")])
@pytest.mark.parametrize("M,N,Kd", [(8192, 768, 3072), (1000, 776, 160), (2048, 200, 64), (777, 96, 2304)])
def test_pp_narrow_tile_forms_with_epilogues(K, bn, form, M, N, Kd):
    """96 / 128-wide ping-pong tiles streaming 64-deep slices (sk64, K % 64 == 0; else the 32-deep form) and
    32-deep slices, with every bf16 epilogue the GPT-2 linears use, against the fp32 reference (ragged M / N
    edges included)."""
    old_bn, old_pp = K.tune_set("pp_bn", bn), K.tune_set("pp", 2)
    old_sk = K.tune_set("pp_sk64", int(form == "sk64"))
    try:
        x, w = rnd(M, Kd), rnd(N, Kd, scale=0.05)
        ref = x.float() @ w.float().t()
        assert rel(K.gemm_nt_ex(x, w), ref) < 1e-2
        bias, res = torch.randn(N, device="cuda"), rnd(M, N)
        assert rel(K.gemm_nt_ex(x, w, bias=bias, res=res), ref + bias + res.float()) < 1e-2
        aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        y = K.gemm_nt_ex(x, w, bias=bias, act=2, aux=aux)
        u = ref + bias
        assert rel(aux, u) < 1e-2
        assert rel(y, F.gelu(aux.float(), approximate="tanh")) < 2e-2
        dg = rnd(M, N)
        g = dg.float()
        t = torch.tanh(0.7978845608 * (g + 0.044715 * g ** 3))
        dgelu = 0.5 * (1 + t) + 0.5 * g * (1 - t * t) * 0.7978845608 * (1 + 3 * 0.044715 * g * g)
        assert rel(K.gemm_nt_ex(x, w, dgelu=dg), ref * dgelu) < 2e-2
    finally:
        K.tune_set("pp_bn", old_bn)
        K.tune_set("pp_sk64", old_sk)
        K.tune_set("pp", old_pp)


@pytest.mark.parametrize("bn", [96, 128, 192, 256, 288])
@pytest.mark.parametrize("M,N,Kd", [(8192, 3072, 768), (4000, 1000, 320), (2048, 8192, 64)])
def test_pp_epilogue_store_slack_and_pairing(K, bn, M, N, Kd):
    """Deferred store drain (tuning pp_epi_slack: buffer-store epilogue, the next items' load waits relaxed) and
    epilogue pairing (pp_epi_pair: both wave groups' epilogues in one barrier interval) give the bits of the
    plain schedule -- several items per block, ragged edges (dropped out-of-range stores), GELU's second output
    -- and match the fp32 reference."""
    old_bn, old_pp = K.tune_set("pp_bn", bn), K.tune_set("pp", 2)
    old_sl, old_pr = K.tune_get("pp_epi_slack"), K.tune_get("pp_epi_pair")
    try:
        x, w = rnd(M, Kd), rnd(N, Kd, scale=0.05)
        bias = torch.randn(N, device="cuda")
        outs = {}
        for sl, pr in ((0, 0), (1, 0), (0, 1), (1, 1)):
            K.tune_set("pp_epi_slack", sl)
            K.tune_set("pp_epi_pair", pr)
            aux = torch.full((M, N), 7.0, device="cuda", dtype=torch.bfloat16)
            y = K.gemm_nt_ex(x, w, bias=bias, act=2, aux=aux)
            outs[sl, pr] = (y, aux, K.gemm_nt_ex(x, w))
        for key in ((1, 0), (0, 1), (1, 1)):
            for a, b in zip(outs[0, 0], outs[key]):
                assert torch.equal(a, b), key
        ref = x.float() @ w.float().t()
        assert rel(outs[1, 1][2], ref) < 1e-2
        assert rel(outs[1, 1][1], ref + bias) < 1e-2
    finally:
        K.tune_set("pp_bn", old_bn)
        K.tune_set("pp", old_pp)
        K.tune_set("pp_epi_slack", old_sl)
        K.tune_set("pp_epi_pair", old_pr)


@pytest.mark.parametrize("splits", [None, 1, 2, 3, 5, 8])
def test_gemm_nt_splitk_uneven(K, splits):
    """The split-K GEMM of the tied LM head's data gradient (K = vocabulary): split counts that do not divide the
    K slices give the first K % s splits one slice more; every split count (and the planned one) must give the
    reference product."""
    M, N, Kd = 512, 768, 50304
    x, w = rnd(M, Kd, scale=0.1), rnd(N, Kd, scale=0.05)
    y = K.gemm_nt_splitk(x, w, splits=splits)
    assert y.shape == (M, N) and y.dtype == torch.bfloat16
    assert rel(y, x.float() @ w.float().t()) < 1e-2


def test_transpose_bf16_multi(K):
    """One launch over many matrices (ragged edges, > 64 entries so the host splits the table)."""
    shapes = [(768, 2304), (3072, 768), (100, 37), (8, 8), (50257, 768)] + [(64 + i, 72 + 3 * i) for i in range(70)]
    srcs = [rnd(r, c) for r, c in shapes]
    dsts = [torch.empty(c, r, device="cuda", dtype=torch.bfloat16) for r, c in shapes]
    K.transpose_bf16_multi(list(zip(srcs, dsts)))
    torch.cuda.synchronize()
    for s_, d_ in zip(srcs, dsts):
        assert torch.equal(d_, s_.t())


@pytest.mark.parametrize("M,N,Kd", [(1000, 776, 1024), (2048, 2048, 64), (4104, 1032, 768), (8192, 3072, 768)])
def test_gemm_large_tile_engine(K, M, N, Kd):
    """Shapes routed to the 256x256 glds engine (K % 64 == 0, enough tiles), incl. ragged M/N edges."""
    x, w = rnd(M, Kd), rnd(N, Kd)
    b = torch.randn(N, device="cuda")
    assert rel(K.gemm_nt(x, w, bias=b), x.float() @ w.float().t() + b) < 1e-2
    assert rel(K.gemm_nt(x, w, out_f32=True), x.float() @ w.float().t()) < 2e-3
    wt = w.t().contiguous()
    assert rel(K.gemm_nn(x, wt), x.float() @ wt.float()) < 1e-2
    g = rnd(M, N)
    dw = torch.zeros(N, Kd, device="cuda")
    K.gemm_tn_acc(g, x, dw)
    assert rel(dw, g.float().t() @ x.float()) < 2e-3


@pytest.mark.parametrize("C,dt", [(3, torch.float32), (1, BF), (10, torch.float32), (16, BF)])
def test_nchw_to_nhwc_pad(K, C, dt):
    x = torch.randn(3, C, 13, 11, device="cuda").to(dt)
    cp = (C + 7) // 8 * 8
    y = K.nchw_to_nhwc(x, cp)
    ref = torch.zeros(3, 13, 11, cp, device="cuda", dtype=BF)
    ref[..., :C] = x.permute(0, 2, 3, 1).to(BF)
    assert torch.equal(y, ref)


@pytest.mark.parametrize("shape", [(2, 8, 8, 64, 256, 1), (2, 56, 56, 64, 256, 1), (3, 7, 7, 512, 2048, 1),
                                   (2, 14, 14, 256, 1024, 1), (2, 9, 9, 64, 64, 3), (2, 28, 28, 128, 128, 3)])
def test_conv_dgrad_masked_residual(K, shape):
    """dx = dgrad(dy) + res * mask (the identity branch of a residual block through the block output's ReLU
    bits), on every engine: the BN backward no longer materialises res * mask."""
    N, H, W, Co, C, R = shape
    pad = R // 2
    x = torch.randn(N, C, H, W, device="cuda", requires_grad=True)
    w = rnd(Co, R, R, C, scale=0.1)
    y = F.conv2d(x, w.float().permute(0, 3, 1, 2), None, 1, pad)
    dy = rnd(*y.permute(0, 2, 3, 1).shape)
    y.backward(dy.float().permute(0, 3, 1, 2))
    res = rnd(N, H, W, C)
    keep = torch.rand(N * H * W, C, device="cuda") > 0.4
    bits = (keep.view(-1, C // 8, 8).to(torch.int32) << torch.arange(8, device="cuda", dtype=torch.int32)).sum(-1)
    mask_u8 = bits.to(torch.uint8).contiguous()
    dx = K.conv_dgrad(dy, w, (N, H, W, C), 1, pad, res=res, res_mask=mask_u8)
    ref = x.grad.permute(0, 2, 3, 1) + res.float() * keep.view(N, H, W, C)
    assert rel(dx, ref) < 1.5e-2




@pytest.mark.parametrize("shape", [(4, 28, 256, 512), (2, 14, 512, 1024), (3, 7, 1024, 2048), (2, 9, 128, 512)])
def test_conv1x1_stride2_dgrad_in_place(K, shape):
    """The ResNet shortcut's data gradient: 1x1 / stride 2, accumulated in place into dx (the ping-pong engine with
    its rows scattered to the even pixels; odd pixels keep dx) against fp32 torch."""
    N, H, C, Ko = shape
    Ho = (H - 1) // 2 + 1
    dy = rnd(N, Ho, Ho, Ko)
    w = rnd(Ko, 1, 1, C, scale=0.05)
    dx0 = rnd(N, H, H, C)
    dx = dx0.clone()
    out = K.conv_dgrad(dy, w, (N, H, H, C), 2, 0, res=dx, out=dx)
    assert out.data_ptr() == dx.data_ptr()
    xi = torch.zeros(N, C, H, H, device="cuda", requires_grad=True)
    y = F.conv2d(xi, w.float().permute(0, 3, 1, 2), None, 2, 0)
    y.backward(dy.float().permute(0, 3, 1, 2))
    ref = xi.grad.permute(0, 2, 3, 1) + dx0.float()
    assert rel(dx, ref) < 1.5e-2
    assert torch.equal(dx[:, 1::2, :, :], dx0[:, 1::2, :, :]) and torch.equal(dx[:, :, 1::2, :], dx0[:, :, 1::2, :])


def test_stat_bins_pool_hands_out_each_slab_once(K):
    """A statistics slab returns to the zeroed free list only once per stat_bins() hand-out: a slab finalized
    twice (or one that never came from the pool) must not be given to two producers."""
    dev = torch.device("cuda")
    s = K.stat_bins(64, dev)
    K.bn_bwd_finalize(s, K.STAT_BINS)
    K.bn_bwd_finalize(s, K.STAT_BINS)           # second finalize: zeroes again, no second release
    foreign = torch.zeros(2 * K.STAT_BINS, 64, device="cuda")
    K.bn_bwd_finalize(foreign, K.STAT_BINS)     # not from the pool: not released into it
    a, b = K.stat_bins(64, dev), K.stat_bins(64, dev)
    assert a.data_ptr() != b.data_ptr() and foreign.data_ptr() not in (a.data_ptr(), b.data_ptr())
    assert not a.any() and not b.any()
