"""Run one ping-pong GEMM configuration repeatedly (rocprofv3 --pmc target).

    python tools/pp_one.py M N K [--bn BN] [--kind nt|nn|wgrad|fwd1x1|fwd1x1pro|dgrad1x1bn] [--iters 20]

The conv kinds run a 1x1 stride-1 conv (M pixels, C = K in, Ko = N out) through the conv API with BN statistics
(fwd1x1), plus the BN-affine+ReLU prologue (fwd1x1pro), or the data gradient with the BN-backward epilogue
(dgrad1x1bn: M pixels, N = C out, K = Ko in); set PDNN_PP_CONV_FWD_K=0 / PDNN_PP_CONV_DGRAD_K=0 to force pp.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pytorch_distributed_nn_amd.ops import kernels as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("M", type=int)
    ap.add_argument("N", type=int)
    ap.add_argument("K", type=int)
    ap.add_argument("--bn", type=int, default=0)
    ap.add_argument("--kind", default="nt")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--trace", action="store_true", help="per-block phase timestamps of one launch")
    a = ap.parse_args()
    r = lambda *s: (torch.rand(*s, device="cuda") * 2 - 1).to(torch.bfloat16)  # noqa: E731
    K.set_pp_mode(2)
    K.set_pp_bn(a.bn)
    if a.kind == "wgrad":
        x, y = r(a.K, a.M), r(a.K, a.N)
        out = torch.zeros(a.M, a.N, device="cuda")
        fn = lambda: K.pp_wgrad(x, y, out)  # noqa: E731
    elif a.kind in ("fwd1x1", "fwd1x1pro"):
        x, w = r(1, a.M, 1, a.K), r(a.N, 1, 1, a.K)
        pro = (torch.rand(a.K, device="cuda") + 0.5, torch.randn(a.K, device="cuda")) if a.kind == "fwd1x1pro" else None
        fn = lambda: K.conv_fwd(x, w, 1, 0, pro=pro, want_stats=True)  # noqa: E731
    elif a.kind == "dgrad1x1bn":
        dy, w, t = r(1, a.M, 1, a.K), r(a.K, 1, 1, a.N), r(1, a.M, 1, a.N)
        v = [torch.rand(a.N, device="cuda") + 0.5 for _ in range(4)]
        fn = lambda: K.conv_dgrad(dy, w, (1, a.M, 1, a.N), 1, 0, bn=(t, *v))  # noqa: E731
    else:
        x, w = r(a.M, a.K), r(a.N, a.K)
        wt = w.t().contiguous()
        fn = (lambda: K.gemm_nt(x, w)) if a.kind == "nt" else (lambda: K.gemm_nn(x, wt))  # noqa: E731
    for _ in range(a.iters):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / a.iters
    if a.trace:
        from pytorch_distributed_nn_amd.ops._backend import lib
        import ctypes
        buf = torch.zeros(2 * 256 * 64, dtype=torch.int64, device="cuda")
        lib().pdnn_set_pp_trace(ctypes.c_void_p(buf.data_ptr()))
        fn()
        torch.cuda.synchronize()
        lib().pdnn_set_pp_trace(None)
        t = buf.view(256, 2, 64).cpu().double() * 10.0     # ns (100 MHz)
        used = t[:, 0, 0] > 0
        t = t[used]
        t0 = t[:, :, 0].min()
        span = (t.max() - t0) / 1e3
        pro = (t[:, :, 1] - t[:, :, 0]).mean() / 1e3
        start = (t[:, :, 0] - t0).mean() / 1e3
        comp, epi = [], []
        prev = t[:, :, 1]
        for i in range(30):
            c, d = t[:, :, 2 + 2 * i], t[:, :, 3 + 2 * i]
            ok = c > 0
            if not ok.any():
                break
            comp.append(((c - prev)[ok]).mean().item() / 1e3)
            epi.append(((d - c)[ok]).mean().item() / 1e3)
            prev = torch.where(ok, d, prev)
        print(f"trace: blocks={int(used.sum())} span={span:.1f}us mean start offset={start:.1f}us prologue={pro:.2f}us "
              f"items={len(comp)} compute/item={sum(comp) / max(1, len(comp)):.2f}us (first {comp[0]:.2f}) "
              f"epilogue/item={sum(epi) / max(1, len(epi)):.2f}us")
    print(f"{a.kind} M={a.M} N={a.N} K={a.K} bn={a.bn} {ms * 1e3:.1f} us {2 * a.M * a.N * a.K / ms / 1e9:.0f} TF/s")


if __name__ == "__main__":
    main()
