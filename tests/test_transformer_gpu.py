"""GPT-2 kernels and fused blocks vs fp32 PyTorch references (BASELINE.json config 4)."""
import copy
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

BF = torch.bfloat16


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


def rel2(a, b):
    a, b = a.float().flatten(), b.float().flatten()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def cos(a, b):
    return F.cosine_similarity(a.float().flatten(), b.float().flatten(), dim=0).item()


@pytest.fixture(scope="module")
def K():
    from pytorch_distributed_nn_amd.ops import _backend, kernels
    assert _backend.available(), "HIP kernel library must load on a GPU box"
    return kernels


def rnd(*s, scale=1.0):
    return (torch.randn(*s, device="cuda") * scale).to(BF)


@pytest.mark.parametrize("R,D", [(300, 768), (64, 128), (257, 1024), (33, 1600)])
def test_layernorm(K, R, D):
    x = rnd(R, D, scale=2.0) + 0.5
    g = torch.randn(D, device="cuda")
    b = torch.randn(D, device="cuda")
    y, mean, rstd = K.layernorm_fwd(x, g, b, 1e-5)
    xr = x.float().requires_grad_(True)
    gr, br = g.clone().requires_grad_(True), b.clone().requires_grad_(True)
    ref = F.layer_norm(xr, (D,), gr, br, 1e-5)
    assert rel(y, ref) < 1e-2
    dy = rnd(R, D)
    dres = rnd(R, D)
    ref.backward(dy.float())
    dx, dg, db = K.layernorm_bwd(dy, x, g, mean, rstd, dres=dres)
    assert rel(dx, xr.grad + dres.float()) < 2e-2
    assert rel(dg, gr.grad) < 1e-3 and rel(db, br.grad) < 1e-3


@pytest.mark.parametrize("B,T,H,causal", [(2, 256, 4, True), (1, 128, 2, False), (2, 1024, 2, True)])
def test_attention_fwd_bwd(K, B, T, H, causal):
    from pytorch_distributed_nn_amd.ops import transformer as TX
    D = 64 * H
    qkv = rnd(B * T, 3 * D)
    y, P, S = TX.attention_fwd(qkv, B, T, H, causal)
    qr = qkv.float().requires_grad_(True)
    ref = TX.attention_reference(qr, B, T, H, causal)
    assert rel2(y, ref) < 1e-2
    dy = rnd(B * T, D)
    ref.backward(dy.float())
    # the causal dP GEMM leaves the scratch's above-diagonal tiles unwritten: poison them (a NaN bit pattern left
    # in reused memory reached dQ through 0 * NaN in the softmax backward's row sums)
    S.fill_(float("nan"))
    dqkv = TX.attention_bwd(dy, qkv, P, B, T, H, causal, dS_buf=S)
    for i, n in enumerate("qkv"):
        a, b = dqkv[:, i * D:(i + 1) * D], qr.grad[:, i * D:(i + 1) * D]
        assert rel2(a, b) < 3e-2, n
        assert cos(a, b) > 0.999, n


def test_gemm_batched_modes(K):
    nb1, nb2, M, N, Kd = 2, 3, 192, 128, 96
    A = rnd(nb1, nb2, M, Kd)
    At = A.transpose(-1, -2).contiguous()
    Bm = rnd(nb1, nb2, N, Kd)
    Bt = Bm.transpose(-1, -2).contiguous()
    ref = A.float() @ Bm.float().transpose(-1, -2)
    sA, sB, sC = (nb2 * M * Kd, M * Kd), (nb2 * N * Kd, N * Kd), (nb2 * M * N, M * N)
    for am, a_, lda in ((0, A, Kd), (1, At, M)):
        for bm, b_, ldb in ((0, Bm, Kd), (1, Bt, N)):
            if am == 1 and bm == 0:
                continue
            for dt in (BF, torch.float32):
                c = torch.empty(nb1, nb2, M, N, device="cuda", dtype=dt)
                K.gemm_batched(a_, lda, sA, am, b_, ldb, sB, bm, c, N, sC, M, N, Kd, (nb1, nb2))
                assert rel(c, ref) < 1e-2, (am, bm, dt)


def test_gemm_gelu_epilogue(K):
    M, N, Kd = 300, 512, 256
    x, w = rnd(M, Kd), rnd(N, Kd, scale=0.1)
    b = torch.randn(N, device="cuda") * 0.1
    u = torch.empty(M, N, device="cuda", dtype=BF)
    h = K.gemm_nt_ex(x, w, bias=b, act=2, aux=u)
    pre = x.float() @ w.float().t() + b
    assert rel(u, pre) < 1e-2
    assert rel(h, F.gelu(pre, approximate="tanh")) < 2e-2
    # backward form: (g . W) * gelu'(u) with W stored [K][N]
    g = rnd(M, 128)
    w2 = rnd(128, N, scale=0.1)
    d = K.gemm_nt_ex(g, w2, dgelu=u, w_kn=True)
    ur = u.float().requires_grad_(True)
    F.gelu(ur, approximate="tanh").backward(g.float() @ w2.float())
    assert rel(d, ur.grad) < 2e-2
    # residual epilogue
    r = rnd(M, N)
    y = K.gemm_nt_ex(x, w, res=r)
    assert rel(y, x.float() @ w.float().t() + r.float()) < 1e-2


def test_embedding(K):
    V, Tm, D, B, T = 1000, 64, 256, 4, 48
    wte, wpe = rnd(V, D), rnd(Tm, D)
    idx = torch.randint(0, V, (B * T,), device="cuda")
    idx[:10] = 7                                     # repeated ids accumulate
    out = K.embedding_fwd(idx, wte, wpe, T)
    pos = torch.arange(T, device="cuda").repeat(B)
    assert rel(out, wte.float()[idx] + wpe.float()[pos]) < 1e-2
    g = rnd(B * T, D)
    dwte = torch.ones(V, D, device="cuda")            # accumulates into existing gradients
    dwpe = torch.ones(Tm, D, device="cuda")
    K.embedding_bwd(idx, g, dwte, dwpe, T)
    rte = torch.ones(V, D, device="cuda").index_add_(0, idx, g.float())
    rpe = torch.ones(Tm, D, device="cuda").index_add_(0, pos, g.float())
    assert rel(dwte, rte) < 1e-4 and rel(dwpe, rpe) < 1e-4


def _tiny(seed=0, **kw):
    from pytorch_distributed_nn_amd.models.gpt2 import build_gpt2
    torch.manual_seed(seed)
    return build_gpt2("gpt2_tiny", **kw)


def test_gpt2_block_matches_reference():
    from pytorch_distributed_nn_amd.ops import transformer as TX
    m = _tiny().cuda()
    blk = m.transformer.h[0]
    B, T, D = 2, 128, 128
    x = (torch.randn(B * T, D, device="cuda")).to(BF)
    ref_blk = copy.deepcopy(blk).float()
    xr = x.float().view(B, T, D).requires_grad_(True)
    ref = ref_blk(xr)
    params, shadows = blk.fused_params()
    xg = x.clone().requires_grad_(True)
    y = TX.GPT2BlockFn.apply(xg, (B, T, 2, 1e-5), shadows, *params)
    assert rel2(y, ref.reshape(B * T, D)) < 2e-2
    g = torch.randn(B * T, D, device="cuda").to(BF)
    ref.backward(g.float().view(B, T, D))
    y.backward(g)
    assert rel2(xg.grad, xr.grad.reshape(B * T, D)) < 5e-2
    for (n, p), (_, pr) in zip(blk.named_parameters(), ref_blk.named_parameters()):
        assert cos(p.grad, pr.grad) > 0.995, n
        assert rel2(p.grad, pr.grad) < 0.08, n


@pytest.mark.parametrize("pp", [0, 2])
def test_gpt2_engines_match_reference(K, pp):
    """GPT-2 (d=256, 4 heads, T=512, B=4: 2048 tokens) loss and every gradient against the fp32 CPU
    reference, with the linears on the ping-pong engine wherever it takes the shape (pp=2) or on the
    register-staged / glds engines only (pp=0)."""
    old = K.set_pp_mode(pp)
    try:
        m = _tiny(n_embd=256, n_head=4, block_size=512).cuda()
        ref = copy.deepcopy(m).float().cpu()
        B, T = 4, 512
        idx = torch.randint(0, m.config.vocab_size, (B, T))
        tgt = torch.randint(0, m.config.vocab_size, (B, T))
        loss = m(idx.cuda(), tgt.cuda())
        lref = ref(idx, tgt)
        assert abs(loss.item() - lref.item()) / lref.item() < 0.01
        loss.backward()
        lref.backward()
        for (n, p), (_, pr) in zip(m.named_parameters(), ref.named_parameters()):
            assert cos(p.grad.cpu(), pr.grad) > 0.99, (pp, n)
            assert rel2(p.grad.cpu(), pr.grad) < 0.1, (pp, n)
    finally:
        K.set_pp_mode(old)


def test_gpt2_tiny_loss_and_grads():
    m = _tiny().cuda()
    ref = copy.deepcopy(m).float().cpu()
    B, T = 4, 128
    idx = torch.randint(0, m.config.vocab_size, (B, T))
    tgt = torch.randint(0, m.config.vocab_size, (B, T))
    loss = m(idx.cuda(), tgt.cuda())
    lref = ref(idx, tgt)
    assert abs(loss.item() - lref.item()) / lref.item() < 0.01
    loss.backward()
    lref.backward()
    for (n, p), (_, pr) in zip(m.named_parameters(), ref.named_parameters()):
        assert cos(p.grad.cpu(), pr.grad) > 0.99, n


def test_gpt2_flat_arena_grads_match_autograd_path():
    """With a flat arena the fused ops accumulate gradients in place (the tied wte: LM head then embedding,
    both into the arena); every gradient must equal the autograd-returned path's."""
    from pytorch_distributed_nn_amd.optim import AdamW, flatten_module
    m = _tiny(seed=3).cuda()
    mf = copy.deepcopy(m)
    flatten_module(mf)
    opt = AdamW(mf.parameters(), lr=1e-3)
    opt.zero_grad()
    B, T = 4, 128
    idx = torch.randint(0, m.config.vocab_size, (B, T), device="cuda")
    tgt = torch.randint(0, m.config.vocab_size, (B, T), device="cuda")
    m(idx, tgt).backward()
    mf(idx, tgt).backward()
    for (n, p), (_, pf) in zip(m.named_parameters(), mf.named_parameters()):
        assert rel2(pf.grad, p.grad) < 1e-3, n


def test_gpt2_side_stream_weight_gradients():
    """tuning gpt2_side_wgrad: the linear weight gradients accumulate into the arena on the side stream beside the
    data-gradient chain (joined at the end of the backward); the gradients must equal the one-stream run's, also
    over two steps (the next step's zero_grad and forward must wait for the side stream)."""
    from pytorch_distributed_nn_amd import tuning
    from pytorch_distributed_nn_amd.optim import AdamW, flatten_module
    B, T = 4, 128
    grads = {}
    for v in (0, 1):
        old = tuning.set("gpt2_side_wgrad", v)
        try:
            torch.manual_seed(0)
            m = _tiny(seed=5).cuda()
            fp = flatten_module(m)
            opt = AdamW(m.parameters(), lr=1e-3)
            g = torch.Generator(device="cuda").manual_seed(9)
            out = []
            for _ in range(2):
                idx = torch.randint(0, m.config.vocab_size, (B, T), device="cuda", generator=g)
                tgt = torch.randint(0, m.config.vocab_size, (B, T), device="cuda", generator=g)
                opt.zero_grad()
                m(idx, tgt).backward()
                out.append(fp.grad.clone())
                opt.step()
            grads[v] = out
        finally:
            tuning.set("gpt2_side_wgrad", old)
    for a, b in zip(grads[0], grads[1]):
        assert rel2(b, a) < 1e-4


def test_gpt2_fused_xent_gradients():
    """tuning xent_fused: the training forward writes softmax - onehot over the logits and the backward scales the
    LM head's products by grad_out / count; gradients (also for a scaled loss) and the loss must match the separate
    passes, and an evaluation forward (no grad) the same loss."""
    from pytorch_distributed_nn_amd import tuning
    from pytorch_distributed_nn_amd.ops import kernels as K
    B, T = 4, 128
    res = {}
    for v in (0, 1):
        old = tuning.set("xent_fused", v)
        try:
            m = _tiny(seed=5).cuda()
            assert m.config.vocab_size % 8 == 0
            g = torch.Generator(device="cuda").manual_seed(9)
            idx = torch.randint(0, m.config.vocab_size, (B, T), device="cuda", generator=g)
            tgt = torch.randint(0, m.config.vocab_size, (B, T), device="cuda", generator=g)
            tgt[0, :5] = -100
            loss = m(idx, tgt)
            (loss * 3.0).backward()
            with torch.no_grad():
                ev = m(idx, tgt)
            res[v] = (loss.detach(), ev, {n: p.grad.clone() for n, p in m.named_parameters()})
        finally:
            tuning.set("xent_fused", old)
    assert K.xent_fwd_grad_ok(torch.empty(8, m.config.vocab_size, device="cuda", dtype=torch.bfloat16))
    assert abs(res[1][0].item() - res[0][0].item()) < 1e-4 * abs(res[0][0].item())
    assert abs(res[1][1].item() - res[0][1].item()) < 1e-4 * abs(res[0][1].item())
    for n, a in res[0][2].items():
        assert rel2(res[1][2][n], a) < 1e-2, n


@pytest.mark.parametrize("mode", [1, 2])
def test_gpt2_prefetched_transposes_track_optimizer_steps(mode):
    """tuning wt_prefetch 1 / 2: the forward refreshes every transposed weight copy in one launch
    (prefetch_weight_t) on the compute / side stream; after each optimizer step the copies must be current
    (version key) and equal W^T of the new shadow."""
    from pytorch_distributed_nn_amd import tuning
    old = tuning.set("wt_prefetch", mode)
    try:
        _prefetch_run()
    finally:
        tuning.set("wt_prefetch", old)


def _prefetch_run():
    from pytorch_distributed_nn_amd.ops import functional as OF
    from pytorch_distributed_nn_amd.optim import AdamW, flatten_module
    m = _tiny(seed=5).cuda()
    flatten_module(m)
    opt = AdamW(m.parameters(), lr=1e-3)
    idx = torch.randint(0, m.config.vocab_size, (2, 128), device="cuda")
    tgt = torch.randint(0, m.config.vocab_size, (2, 128), device="cuda")
    for _ in range(3):
        opt.zero_grad()
        loss = m(idx, tgt)
        torch.cuda.synchronize()
        for p in m._t_weights():
            ver, wt = p._pdnn_shadow_t
            assert ver == OF._t_version(p)
            assert torch.equal(wt, OF.weight_bf16(p).t())
        loss.backward()
        opt.step()


def test_gpt2_tiny_trains():
    from pytorch_distributed_nn_amd.optim import AdamW, flatten_module
    m = _tiny(seed=1).cuda()
    flatten_module(m)
    opt = AdamW(m.parameters(), lr=3e-3, weight_decay=0.0)
    idx = torch.randint(0, 64, (4, 129), device="cuda")     # small vocabulary subset: learnable
    x, y = idx[:, :-1].contiguous(), idx[:, 1:].contiguous()
    first = None
    for _ in range(30):
        opt.zero_grad()
        loss = m(x, y)
        loss.backward()
        opt.step()
        first = first if first is not None else loss.item()
    assert math.isfinite(loss.item()) and loss.item() < 0.7 * first


@pytest.mark.parametrize("causal", [True, False])
def test_flash_attention_growing_scores(K, causal):
    """Scores whose row maximum keeps growing (and jumps) across key tiles: the forward's lazy rescale (the
    running maximum moves only past a 2^8 margin) must give the same output and log-sum-exp."""
    from pytorch_distributed_nn_amd.ops import transformer as TX
    B, T, H = 1, 1024, 2
    D = 64 * H
    g = torch.Generator(device="cuda").manual_seed(7)
    qkv = torch.randn(B * T, 3 * D, device="cuda", generator=g)
    ramp = torch.linspace(0.2, 6.0, T, device="cuda").view(T, 1)
    ramp[600:] += 4.0                                        # a jump well past the margin
    qkv[:, D:2 * D] *= ramp                                  # later keys score higher
    qkv[:, :D] *= 2.0
    qkv = qkv.to(torch.bfloat16)
    y, lse2 = K.flash_attn_fwd(qkv, B, T, H, 0.125, causal)
    ref = TX.attention_reference(qkv.float(), B, T, H, causal)
    assert rel2(y, ref) < 1e-2
    q, k, _ = qkv.float().view(B, T, 3, H, 64).permute(2, 0, 3, 1, 4)
    s = (q @ k.transpose(-1, -2)) * 0.125
    if causal:
        s = s.masked_fill(torch.ones(T, T, device="cuda", dtype=torch.bool).triu(1), float("-inf"))
    assert rel(lse2, torch.logsumexp(s, -1) * 1.4426950408889634) < 1e-3


@pytest.mark.parametrize("B,T,H,causal", [(2, 256, 3, True), (1, 128, 2, False), (2, 1024, 2, True), (1, 384, 1, False)])
def test_flash_attention(K, B, T, H, causal):
    from pytorch_distributed_nn_amd.ops import transformer as TX
    D = 64 * H
    qkv = rnd(B * T, 3 * D)
    y, lse2 = K.flash_attn_fwd(qkv, B, T, H, 0.125, causal)
    qr = qkv.float().requires_grad_(True)
    ref = TX.attention_reference(qr, B, T, H, causal)
    assert rel2(y, ref) < 1e-2
    # log-sum-exp (base 2, scaled domain) vs reference
    q, k, _ = qkv.float().view(B, T, 3, H, 64).permute(2, 0, 3, 1, 4)
    s = (q @ k.transpose(-1, -2)) * 0.125
    if causal:
        s = s.masked_fill(torch.ones(T, T, device="cuda", dtype=torch.bool).triu(1), float("-inf"))
    assert rel(lse2, torch.logsumexp(s, -1) * 1.4426950408889634) < 1e-3
    dy = rnd(B * T, D)
    ref.backward(dy.float())
    dqkv = K.flash_attn_bwd(qkv, y, dy, lse2, B, T, H, 0.125, causal)
    for i, n in enumerate("qkv"):
        a, b = dqkv[:, i * D:(i + 1) * D], qr.grad[:, i * D:(i + 1) * D]
        assert rel2(a, b) < 3e-2, n
        assert cos(a, b) > 0.999, n
