"""Attention kernels at the GPT-2 shape, a few launches each (driver for rocprofv3 --pmc runs)."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_nn_amd.ops import kernels as K  # noqa: E402

B, T, H = 8, 1024, 12
causal = (sys.argv[1] if len(sys.argv) > 1 else "1") == "1"
qkv = (torch.randn(B * T, 3 * H * 64, device="cuda") * 0.5).bfloat16()
sc = 1 / math.sqrt(64)
for _ in range(3):
    out, lse = K.flash_attn_fwd(qkv, B, T, H, sc, causal)
    dq = K.flash_attn_bwd(qkv, out, torch.ones_like(out), lse, B, T, H, sc, causal)
torch.cuda.synchronize()
