"""Every entry of the dispatch table (csrc/kernels/tuning.h + pytorch_distributed_nn_amd/tuning.py) run at
its alternative values: the kernels it routes to must still match the fp32 torch reference (VERDICT r2 #8:
one table instead of per-knob environment variables, each entry exercised)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
BF = torch.bfloat16

# kernel-side entries -> alternative values
ALT = {"glds": [0, 2], "pp": [0, 2], "pp_bn": [96, 128, 192, 288], "conv3x3_force": [1], "pp_dgrad_bn_k": [512, 1 << 20],
       "comm_cus": [0, 64], "pp_sk64": [0], "pp_epi_slack": [0, 1], "pp_epi_pair": [0], "pp_conv_fwd_c": [128, 1 << 20], "stem_wgrad_blocks": [512],
       "attn_delta_in_dq": [0], "attn_bwd_wide": [0, 1]}


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


def _battery(K):
    g = torch.Generator(device="cuda").manual_seed(0)
    rn = lambda *s, sc=1.0: (torch.randn(*s, device="cuda", generator=g) * sc).to(BF)   # noqa: E731
    x, w = rn(1000, 512), rn(776, 512, sc=0.05)
    assert rel(K.gemm_nt(x, w), x.float() @ w.float().t()) < 1e-2
    # linear weight gradient on the planned (tile width, K-splits), fused bias column sums
    xg, yg = rn(4096, 768), rn(4096, 256)
    out, bias = torch.zeros(768, 256, device="cuda"), torch.zeros(768, device="cuda")
    K.pp_wgrad(xg, yg, out, rowsum=bias)
    assert rel(out, xg.float().t() @ yg.float()) < 1e-3 and rel(bias, xg.float().sum(0)) < 1e-3
    out2 = torch.zeros(768, 256, device="cuda")
    K.pp_wgrad(xg, yg, out2, plan_cus=64)        # side-stream plan (fewer splits)
    assert rel(out2, xg.float().t() @ yg.float()) < 1e-3
    for (N, H, C, Ko, R, st, pad) in [(2, 14, 128, 128, 3, 1, 1), (2, 14, 128, 128, 3, 2, 1), (2, 14, 64, 256, 1, 1, 0),
                                      (2, 8, 256, 512, 1, 1, 0), (2, 14, 128, 512, 1, 1, 0), (2, 8, 512, 128, 1, 1, 0), (3, 7, 512, 512, 3, 1, 1),
                                      (4, 14, 256, 1024, 1, 1, 0), (8, 14, 128, 512, 1, 1, 0)]:
        xi = torch.randn(N, C, H, H, device="cuda", generator=g, requires_grad=True)
        wk = rn(Ko, R, R, C, sc=0.05)
        y = F.conv2d(xi, wk.float().permute(0, 3, 1, 2), None, st, pad)
        dy = rn(*y.permute(0, 2, 3, 1).shape)
        y.backward(dy.float().permute(0, 3, 1, 2))
        xn = xi.detach().permute(0, 2, 3, 1).contiguous().to(BF)
        yk, slab = K.conv_fwd(xn, wk, st, pad, want_stats=True)
        yr = F.conv2d(xn.float().permute(0, 3, 1, 2), wk.float().permute(0, 3, 1, 2), None, st, pad).permute(0, 2, 3, 1)
        assert rel(yk, yr) < 1.5e-2
        assert torch.allclose(slab.view(-1, 2, Ko).sum(0)[0], yk.float().reshape(-1, Ko).sum(0), rtol=1e-3,
                              atol=1e-2 * yk.float().abs().max().item())
        assert rel(K.conv_dgrad(dy, wk, (N, H, H, C), st, pad), xi.grad.permute(0, 2, 3, 1)) < 1.5e-2
        if R == 1 and st == 1:
            # the BN-backward epilogue form of the data gradient (pp_dgrad_bn_k routes it between engines)
            t = rn(*xn.shape)
            mean, inv = torch.randn(C, device="cuda", generator=g) * 0.1, torch.rand(C, device="cuda", generator=g) + 0.5
            bsc, bsh = torch.rand(C, device="cuda", generator=g) + 0.5, torch.randn(C, device="cuda", generator=g) * 0.3
            gm, slab = K.conv_dgrad(dy, wk, (N, H, H, C), 1, 0, bn=(t, mean, inv, bsc, bsh))
            z = t.float() * bsc + bsh
            gm_ref = xi.grad.permute(0, 2, 3, 1).to(BF).float() * (z > 0)
            sure = z.abs() > 1e-4
            assert rel(gm.float() * sure, gm_ref * sure) < 1.5e-2
            s0 = slab.view(-1, 2, C).sum(0)[0]
            assert torch.allclose(s0, gm_ref.reshape(-1, C).sum(0), rtol=1e-2, atol=5e-2 + 1e-3 * gm_ref.abs().sum(dim=(0, 1, 2)).max().item())
        dw = K.conv_wgrad(xn, dy, R, R, st, pad)
        dwr = torch.nn.grad.conv2d_weight(xn.float().permute(0, 3, 1, 2), wk.permute(0, 3, 1, 2).shape,
                                          dy.float().permute(0, 3, 1, 2), st, pad).permute(0, 2, 3, 1)
        assert rel(dw, dwr) < 1e-2


@pytest.fixture(scope="module")
def K():
    from pytorch_distributed_nn_amd.ops import kernels, _backend
    assert _backend.available()
    return kernels


def test_table_lists_every_entry(K):
    keys = {k for k, *_ in K.tune_table()}
    assert keys == set(ALT)
    for k, v, d, doc in K.tune_table():
        assert v == d and doc, k          # the test process runs the defaults


@pytest.mark.parametrize("key,value", [(k, v) for k, vs in ALT.items() for v in vs])
def test_kernel_entry_alternatives(K, key, value):
    old = K.tune_set(key, value)
    old_world = K.set_comm_world(4) if key == "comm_cus" else None      # the entry acts only at world > 1
    try:
        _battery(K)
    finally:
        K.tune_set(key, old)
        if old_world is not None:
            K.set_comm_world(old_world)


def test_comm_world_reserves_cus_for_rccl(K):
    """VERDICT r4 #3b: while a multi-rank process group is live the persistent grids leave comm_cus CUs (whole
    XCDs' worth, multiple of 8) to RCCL's channel blocks; at world 1 they fill the chip.  The persistent GEMMs and
    convs must stay exact under the smaller grids (a persistent grid that assumed one block per CU would skip
    tiles)."""
    hw = torch.cuda.get_device_properties(0).multi_processor_count
    assert K.grid_cus() == hw // 8 * 8
    old = K.set_comm_world(8)
    try:
        assert K.grid_cus() == (hw - K.tune_get("comm_cus")) // 8 * 8
        prev = K.tune_set("comm_cus", 21)
        try:
            assert K.grid_cus() == (hw - 21) // 8 * 8
            _battery(K)
        finally:
            K.tune_set("comm_cus", prev)
    finally:
        K.set_comm_world(old)
    assert K.grid_cus() == hw // 8 * 8


def _resnet_grads(arch="resnet50"):
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.ops import functional as OF
    from pytorch_distributed_nn_amd.optim import flatten_module
    torch.manual_seed(0)
    m = build_model(arch).cuda()
    fp = flatten_module(m)
    g = torch.Generator().manual_seed(5)
    x = torch.randn(4, 3, 64, 64, generator=g).cuda().to(BF)
    y = torch.randint(0, 1000, (4,), generator=g).cuda()
    fp.zero_grad()
    OF.cross_entropy(m(x), y).backward()
    torch.cuda.synchronize()
    return fp.grad.clone()


@pytest.mark.parametrize("key,arch", [("side_wgrad", "resnet50"), ("wide1x1_dgrad", "resnet50"),
                                      ("conv3x3", "resnet50"), ("panel1x1", "resnet50"), ("side_wgrad", "resnet18"),
                                      ("a2_fold", "resnet50")])
# (the stem entry is compared at the StemFn level in tests/test_stem_gpu.py: a 1-ulp flip in the stem output
# -- the NCHW kernel's different summation order -- is amplified by this 4-image net's tiny BatchNorm batches
# into O(1) gradient differences; modes 0 and 1 are bitwise equal, gpurun_out/r3_23)
def test_python_entry_alternatives(K, key, arch):
    """The model-level switches change only the schedule / kernel choice: same gradients (bf16 noise)."""
    from pytorch_distributed_nn_amd import tuning
    base = _resnet_grads(arch)
    # conv3x3 / panel1x1: the routers' own switches (set_conv3x3_mode / set_panel_mode), not table entries
    # a2_fold: the 64x64 test images are below the default's pixel threshold, so compare off (0) against everywhere (2)
    if key == "a2_fold":
        tuning.set(key, 2)
        base = _resnet_grads(arch)
        tuning.set(key, tuning.DEFAULTS[key])
    old = tuning.set(key, 0) if key in tuning.DEFAULTS else None
    if key == "conv3x3":
        K.set_conv3x3_mode(0)
    if key == "panel1x1":
        K.set_panel_mode(0)
    try:
        alt = _resnet_grads(arch)
    finally:
        if old is not None:
            tuning.set(key, old)
        K.set_conv3x3_mode(1)
        K.set_panel_mode(1)
    cos = torch.nn.functional.cosine_similarity(base, alt, dim=0).item()
    assert cos > 0.995, (key, cos)
