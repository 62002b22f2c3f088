"""Per-tile overhead vs per-slice cost of the ping-pong engine: plain bf16 GEMMs at fixed M x N over K
(one tile round at N = 768 / 96-wide, two at N = 3072 / 192-wide), us per call, ours vs torch."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pytorch_distributed_nn_amd.ops import kernels as K  # noqa: E402
from gpt2_gemms import timeit  # noqa: E402

for M, N in [(8192, 768), (8192, 3072)]:
    for Kd in (256, 512, 768, 1536, 3072, 6144):
        x = ((torch.rand(M, Kd, device="cuda") * 2 - 1)).to(torch.bfloat16)
        w = ((torch.rand(N, Kd, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
        out = {"M": M, "N": N, "K": Kd, "ours": timeit(lambda: K.gemm_nt_ex(x, w)), "torch": timeit(lambda: x @ w.t())}
        print(json.dumps(out), flush=True)
