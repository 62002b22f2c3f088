"""OOB / determinism probe of the stride-2 dgrad kernel at the shapes of the round-6 rehearsal failure (ResNet-50,
64x64 input, batch 4) and bs 256: guard zones around dx and the statistics slab, 40 repeats compared bitwise."""
import sys

import torch

sys.path.insert(0, ".")
from pytorch_distributed_nn_amd import tuning  # noqa: E402
from pytorch_distributed_nn_amd.ops import kernels as K  # noqa: E402

BF = torch.bfloat16
tuning.set("s2_halo", 1)
PAIR = int(sys.argv[1]) if len(sys.argv) > 1 else 0
torch.manual_seed(0)
bad = 0
for (N, H, W, C) in [(4, 16, 16, 128), (4, 8, 8, 256), (4, 4, 4, 512), (256, 56, 56, 128), (256, 28, 28, 256),
                     (256, 14, 14, 512)]:
    w = (torch.randn(C, 3, 3, C, device="cuda") * 0.05).to(BF)
    dy = torch.randn(N, H // 2, W // 2, C, device="cuda").to(BF)
    t = torch.randn(N, H, W, C, device="cuda").to(BF)
    mean, inv = torch.randn(C, device="cuda") * 0.1, torch.rand(C, device="cuda") + 0.5
    msc, msh = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.3
    wt = K.conv3x3_flip(w)
    G = 1 << 16
    n = N * H * W * C
    big = torch.full((n + 2 * G,), 0x7FC1, dtype=torch.int16, device="cuda")      # NaN-pattern guards
    sbig = torch.full((2 * 64 * C + 2 * G,), 777.0, device="cuda")
    ref = None
    for it in range(40):
        big[G:G + n].zero_()
        sbig[G:G + 2 * 64 * C].zero_()
        dx = big[G:G + n].view(BF).view(N, H, W, C)
        slab = sbig[G:G + 2 * 64 * C].view(2 * 64, C)
        K.call("pdnn_conv3x3s2", K.ptr(dy), K.ptr(wt), K.ptr(dx), N, H, W, C, C, 1, K.ptr(slab), K.ptr(t), K.ptr(mean),
               K.ptr(inv), K.ptr(msc), K.ptr(msh), None, None, None, None, None, None, None, None, None, PAIR, K.stream())
        torch.cuda.synchronize()
        g_ok = bool((big[:G] == 0x7FC1).all() and (big[G + n:] == 0x7FC1).all())
        s_ok = bool((sbig[:G] == 777.0).all() and (sbig[G + 2 * 64 * C:] == 777.0).all())
        cur = (dx.clone(), slab.sum(0).clone())
        if ref is None:
            ref = cur
        same = torch.equal(cur[0], ref[0])
        sdiff = (cur[1] - ref[1]).abs().max().item()
        if not (g_ok and s_ok and same) or sdiff > 1e-3 * ref[1].abs().max().item():
            bad += 1
            print("MISMATCH", (N, H, W, C), it, g_ok, s_ok, same, sdiff, flush=True)
    print("shape", (N, H, W, C), "done", flush=True)
print("bad", bad)
