"""Single-GEMM driver for PMC counter runs: python tools/exp_pmc.py M N K [ours|torch]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_nn_amd.ops import kernels as K  # noqa: E402

M, N, Kd = (int(v) for v in sys.argv[1:4])
which = sys.argv[4] if len(sys.argv) > 4 else "ours"
x = torch.randn(M, Kd, device="cuda").bfloat16()
w = torch.randn(N, Kd, device="cuda").bfloat16()
for _ in range(5):
    y = K.gemm_nt(x, w) if which == "ours" else x @ w.t()
torch.cuda.synchronize()
