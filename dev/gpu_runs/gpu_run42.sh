#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/run42
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python bench.py --model resnet152 --steps 10 --warmup 5 > $O/r152_bf16.log 2>&1 || exit $?
$T 300 python bench.py --model resnet152 --steps 10 --warmup 5 --fp8 > $O/r152_fp8.log 2>&1 || exit $?
$T 300 python bench.py --model gpt2_small --fp8 > $O/gpt2_fp8.log 2>&1 || exit $?
$T 200 python -c "
import torch, time
a = torch.randn(8192, 768, device='cuda').to(torch.float8_e4m3fn)
b = torch.randn(3072, 768, device='cuda').to(torch.float8_e4m3fn)
s = torch.tensor(1.0, device='cuda')
for dt in (torch.bfloat16,):
    y = torch._scaled_mm(a, b.t(), scale_a=s, scale_b=s, out_dtype=dt)
    torch.cuda.synchronize(); t=time.perf_counter()
    for _ in range(50): y = torch._scaled_mm(a, b.t(), scale_a=s, scale_b=s, out_dtype=dt)
    torch.cuda.synchronize(); dtm=(time.perf_counter()-t)/50
    print('scaled_mm fc fwd', dtm*1e6, 'us', 2*8192*3072*768/dtm/1e12, 'TF')
" > $O/scaled_mm.log 2>&1 || exit $?
