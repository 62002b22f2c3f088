import sys, os, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from pytorch_distributed_nn_amd.ops import kernels as K
def timeit(fn, it=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(it): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / it
N, H, W, C, Ko = 256, 56, 56, 64, 256
x = torch.randn(N, H, W, C, device="cuda").bfloat16()
w = (torch.randn(Ko, 1, 1, C, device="cuda") * 0.05).bfloat16()
print("conv stats", timeit(lambda: K.conv_fwd(x, w, 1, 0, want_stats=True)))
print("conv nostats", timeit(lambda: K.conv_fwd(x, w, 1, 0, want_stats=False)))
x2 = x.view(-1, C); w2 = w.view(Ko, C)
print("gemm_nt", timeit(lambda: K.gemm_nt(x2, w2)))
y = torch.empty(N * H * W, Ko, device="cuda").bfloat16()
print("torch copy 411MB write (fill)", timeit(lambda: y.fill_(1.0)))
print("torch matmul", timeit(lambda: x2 @ w2.t()))
xc = x.permute(0, 3, 1, 2); wc = w.permute(0, 3, 1, 2)
import torch.nn.functional as F
print("miopen conv", timeit(lambda: F.conv2d(xc, wc)))
for ss in (0, 1):
    K.set_staged_store(ss)
    print("staged", ss, "gemm_nt", timeit(lambda: K.gemm_nt(x2, w2)))
