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
