"""Cost of each ping-pong GEMM epilogue on the GPT-2 shapes (what the fused linears add over a plain GEMM).

python dev/probes/epi_cost.py  -> one JSON line per shape: us per variant"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def timeit(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / iters * 1e3, 1)


def main():
    from pytorch_distributed_nn_amd.ops import kernels as K
    for name, M, N, Kd in [("fc", 8192, 3072, 768), ("proj", 8192, 768, 768), ("fc2", 8192, 768, 3072),
                           ("qkv", 8192, 2304, 768)]:
        x = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
        w = (torch.randn(N, Kd, device="cuda") * 0.05).to(torch.bfloat16)
        b = torch.randn(N, device="cuda")
        aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        r = torch.randn(M, N, device="cuda").to(torch.bfloat16)
        out = {"shape": name}
        out["plain"] = timeit(lambda: K.gemm_nt_ex(x, w))
        out["bias"] = timeit(lambda: K.gemm_nt_ex(x, w, bias=b))
        out["bias_relu"] = timeit(lambda: K.gemm_nt_ex(x, w, bias=b, act=1))
        out["bias_gelu_noaux"] = timeit(lambda: K.gemm_nt_ex(x, w, bias=b, act=2))
        out["bias_gelu_aux"] = timeit(lambda: K.gemm_nt_ex(x, w, bias=b, act=2, aux=aux))
        out["res"] = timeit(lambda: K.gemm_nt_ex(x, w, res=r))
        out["bias_res"] = timeit(lambda: K.gemm_nt_ex(x, w, bias=b, res=r))
        out["dgelu"] = timeit(lambda: K.gemm_nt_ex(x, w, dgelu=r))
        out["torch"] = timeit(lambda: x @ w.t())
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
