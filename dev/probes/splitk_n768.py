"""GPT-2's N = 768 GEMMs (fc2 / fc dgrad K = 3072, qkv dgrad K = 2304, proj K = 768): the one-round 256 x 96
tiles of the ping-pong engine vs 256 x 256 tiles with the reduction split over work items (fp32 slabs + a
reduce kernel), vs hipBLASLt.  us per call."""
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
    for name, M, N, Kd in [("fc2", 8192, 768, 3072), ("qkv_dgrad", 8192, 768, 2304), ("proj", 8192, 768, 768)]:
        x = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
        w = (torch.randn(N, Kd, device="cuda") * 0.05).to(torch.bfloat16)
        ref = (x.float() @ w.float().t())
        out = {"shape": name, "torch": timeit(lambda: x @ w.t()), "pp_auto": timeit(lambda: K.gemm_nt_ex(x, w))}
        for bn in (128, 192, 256):
            old = K.tune_set("pp_bn", bn)
            out[f"pp_bn{bn}"] = timeit(lambda: K.gemm_nt_ex(x, w))
            K.tune_set("pp_bn", old)
        for s in (2, 3, 4, 6):
            if (Kd // 32) % s:
                continue
            ws = torch.empty(s * (M * N + 64), device="cuda")
            y = K.gemm_nt_splitk(x, w, splits=s, ws=ws)
            err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
            out[f"splitk{s}"] = timeit(lambda: K.gemm_nt_splitk(x, w, splits=s, ws=ws))
            out[f"splitk{s}_err"] = round(err, 5)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
