"""Time the fused attention kernels (attention.hip) alone at GPT-2 shapes vs torch SDPA (reference point).

    python tools/bench_attn.py            # one JSON line per config
"""
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from pytorch_distributed_nn_amd.ops import kernels as K  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3       # us


def main():
    for B, T, H, causal in [(8, 1024, 12, True), (8, 1024, 12, False), (2, 4096, 12, True), (32, 1024, 12, True)]:
        D = H * 64
        qkv = (torch.randn(B * T, 3 * D, device="cuda") * 0.5).to(torch.bfloat16)
        sc = 1 / math.sqrt(64)
        out, lse = K.flash_attn_fwd(qkv, B, T, H, sc, causal)
        do = torch.randn_like(out)
        fl = 4 * B * H * T * T * 64 * (0.5 if causal else 1.0)
        r = {"B": B, "T": T, "H": H, "causal": causal}
        r["fwd_us"] = timeit(lambda: K.flash_attn_fwd(qkv, B, T, H, sc, causal))
        r["bwd_us"] = timeit(lambda: K.flash_attn_bwd(qkv, out, do, lse, B, T, H, sc, causal))
        r["fwd_tf"] = fl / r["fwd_us"] / 1e6
        r["bwd_tf"] = 2.5 * fl / r["bwd_us"] / 1e6
        q, k, v = (qkv.view(B, T, 3, H, 64).permute(2, 0, 3, 1, 4))
        try:
            r["sdpa_fwd_us"] = timeit(lambda: F.scaled_dot_product_attention(q, k, v, is_causal=causal))
        except Exception as ex:      # noqa: BLE001
            r["sdpa_err"] = repr(ex)[:100]
        print(json.dumps({k2: (round(v2, 2) if isinstance(v2, float) else v2) for k2, v2 in r.items()}), flush=True)


if __name__ == "__main__":
    main()
