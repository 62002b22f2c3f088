"""Statistics-bins probe: conv_dgrad's fused BN-backward sums and conv_fwd's BN statistics under every engine
setting, against torch sums (round-5 atomic bins)."""
import sys
import torch
sys.path.insert(0, ".")
from pytorch_distributed_nn_amd.ops import kernels as K  # noqa: E402

BF = torch.bfloat16
torch.manual_seed(0)


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-9)).item()


for glds, staged, pp in [(1, 1, 1), (0, 1, 0), (0, 0, 0), (2, 1, 0), (1, 1, 2)]:
    K.set_glds_mode(glds); K.set_staged_store(staged); K.set_pp_mode(pp)
    for (N, H, W, C, Ko, R, st, pad) in [(2, 14, 14, 128, 128, 3, 2, 1), (2, 9, 9, 64, 128, 3, 1, 1), (2, 8, 8, 256, 64, 1, 1, 0)]:
        w = (torch.randn(Ko, R, R, C, device="cuda") * 0.1).to(BF)
        Ho, Wo = K.conv_out_hw(H, W, R, R, st, pad)
        dy = torch.randn(N, Ho, Wo, Ko, device="cuda").to(BF)
        t = torch.randn(N, H, W, C, device="cuda").to(BF) + 0.3
        mean, inv = torch.randn(C, device="cuda") * 0.1, torch.rand(C, device="cuda") + 0.5
        sc, sh = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.3
        gm, slab = K.conv_dgrad(dy, w, (N, H, W, C), st, pad, bn=(t, mean, inv, sc, sh))
        s = slab.view(-1, 2, C).sum(0)
        gmf = gm.float().reshape(-1, C)
        xh = ((t.float() - mean) * inv).reshape(-1, C)
        nz = (slab.view(-1, 2, C)[:, 0].abs().sum(1) > 0).sum().item()
        print(f"eng={glds,staged,pp} dgrad {N,H,W,C,Ko,R,st,pad}: sum rel {rel(s[0], gmf.sum(0)):.2e} "
              f"xhat rel {rel(s[1], (gmf * xh).sum(0)):.2e} nonzero bins {nz}", flush=True)
        x = torch.randn(N, H, W, C, device="cuda").to(BF)
        y, sl = K.conv_fwd(x, w, st, pad, want_stats=True)
        yf = y.float().reshape(-1, Ko)
        s2 = sl.view(-1, 2, Ko).sum(0)
        print(f"     fwd: sum rel {rel(s2[0], yf.sum(0)):.2e} sq rel {rel(s2[1], (yf * yf).sum(0)):.2e}", flush=True)
