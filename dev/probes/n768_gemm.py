"""GPT-2's N = 768 GEMMs on the in-tree ping-pong engine vs torch (hipBLASLt): 20 calls each of fc2 (8192 x 768 x
3072), qkv dgrad (x 2304) and proj (x 768), for kernel traces / PMC passes (kernel names tell the vendor tiles)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pytorch_distributed_nn_amd.ops import kernels as K  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "both"
shapes = [("fc2", 8192, 768, 3072), ("qkv_dgrad", 8192, 768, 2304), ("proj", 8192, 768, 768)]
if len(sys.argv) > 2:
    shapes = [s_ for s_ in shapes if s_[0] == sys.argv[2]]
for name, M, N, Kd in shapes:
    x = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
    w = (torch.randn(N, Kd, device="cuda") * 0.05).to(torch.bfloat16)
    for _ in range(20):
        if which in ("both", "ours"):
            K.gemm_nt_ex(x, w)
        if which in ("both", "torch"):
            torch.matmul(x, w.t())
    torch.cuda.synchronize()
print("ok")
