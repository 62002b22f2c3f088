"""LayerNorm backward grid sweep on GPT-2's shape (8192 x 768, with the residual-gradient add): rows per block x
block cap, us per call including its bins finalize.  The two tuning entries it sets (ln_bwd_rows / ln_bwd_blocks)
existed only for this sweep (gpurun_out/r6_19, profiles/layernorm_bwd_grid_r6.txt) and were removed with the
defaults kept; re-add them to csrc/kernels/tuning.h (pdnn_layernorm_bwd_blocks) to rerun it."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pytorch_distributed_nn_amd.ops import kernels as K  # noqa: E402


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / iters * 1e3, 2)


def main():
    R, D = 8192, 768
    x = torch.randn(R, D, device="cuda").to(torch.bfloat16)
    dy = torch.randn(R, D, device="cuda").to(torch.bfloat16)
    dres = torch.randn(R, D, device="cuda").to(torch.bfloat16)
    g, b = torch.rand(D, device="cuda") + 0.5, torch.randn(D, device="cuda")
    _, m, r = K.layernorm_fwd(x, g, b, 1e-5)
    ref = K.layernorm_bwd(dy, x, g, m, r, dres=dres)
    out = {"fwd": timeit(lambda: K.layernorm_fwd(x, g, b, 1e-5))}
    for rows in (16, 8, 4, 2):
        for cap in (512, 1024, 2048, 4096):
            o1, o2 = K.tune_set("ln_bwd_rows", rows), K.tune_set("ln_bwd_blocks", cap)
            dx, dg, db = K.layernorm_bwd(dy, x, g, m, r, dres=dres)
            assert torch.equal(dx, ref[0])
            assert torch.allclose(dg, ref[1], rtol=1e-4, atol=1e-3) and torch.allclose(db, ref[2], rtol=1e-4, atol=1e-3)
            out[f"r{rows}_c{cap}"] = timeit(lambda: K.layernorm_bwd(dy, x, g, m, r, dres=dres))
            K.tune_set("ln_bwd_rows", o1)
            K.tune_set("ln_bwd_blocks", o2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
